"""GPU: the second DGKS refinement (SRC/dsaitr.f:753-781) in the free-running
driver, where it is not enqueued per step: the DGKS1 finalize parks the cycle
(st.abort = 2) and the host runs update + finalize for that step, then resumes.

The refinement is rare on real problems (0 of the golden fixtures take it), so
the test hook AHIP_FORCE_DGKS2=1 makes every step take it.  Both drivers must
then produce the same solve bit for bit -- the free-running one resolving it on
the host at every step, the RCI one in-stream (gated kernels) -- and the result
must still be the reference's (the extra sweep only re-orthogonalises again).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _solve(tmp_path, fixture, how, force):
    out = tmp_path / f"{fixture}_{how}_{int(force)}.npz"
    env = dict(os.environ, AHIP_FORCE_DGKS2="1" if force else "0")
    r = subprocess.run([sys.executable, os.path.join(HERE, "dgks_worker.py"), fixture, how, str(out)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return dict(np.load(out))


@pytest.mark.parametrize("fixture", ["g4_banded", "g3_anderson3d"])
def test_forced_second_refinement_free_vs_rci(tmp_path, golden, fixture):
    g = golden(fixture)
    free = _solve(tmp_path, fixture, "free", True)
    rci = _solve(tmp_path, fixture, "rci", True)
    assert int(free["nitref"]) > 0 and int(free["nitref"]) == int(rci["nitref"])
    for k in ("iters", "nopx", "nrorth", "info"):
        assert int(free[k]) == int(rci[k]), k
    np.testing.assert_array_equal(free["d"], rci["d"])
    np.testing.assert_array_equal(free["z"], rci["z"])
    # still the reference's solve
    np.testing.assert_allclose(np.sort(free["d"]), np.sort(g["d"]), rtol=0,
                               atol=max(1e-10, 10 * float(g["tol"])) * np.abs(g["d"]).max())
    assert int(free["iters"]) == int(g["iparam"][2])


def test_unforced_free_run_takes_no_second_refinement(tmp_path):
    r = _solve(tmp_path, "g4_banded", "free", False)
    assert int(r["nitref"]) == 0
