"""GPU: folded Lanczos steps (sym.cpp saitr, kernels.hip k_fold_dots) -- the
free-running dsaupd engine applies step j-1's DGKS sweep inside step j's first
pass over V and rebuilds A r' from the SpMV of the pre-sweep residual with the
Lanczos relation (A V s = V (T s) + s_j r').  That is an O(eps*|s|)
re-association of SRC/dsaitr.f:680-692 + the next step's OP, not a different
algorithm: the solve must take the reference's restart cycles, OP*x count and
re-orthogonalisation count, and give its Ritz values and vectors.

AHIP_FOLD=0 selects the unfolded (chained) engine as the comparison; the env
is read once per process, hence the subprocess workers.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import matrices as M
from oracle import ref

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _solve_env(tmp_path, fixture, extra, how="free"):
    tag = "_".join("%s%s" % kv for kv in sorted(extra.items()))
    out = tmp_path / f"{fixture}_{how}_{tag}.npz"
    env = dict(os.environ, AHIP_FORCE_DGKS2="0")
    env.update(extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "dgks_worker.py"), fixture, how, str(out)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return dict(np.load(out))


def _solve(tmp_path, fixture, fold):
    return _solve_env(tmp_path, fixture, dict(AHIP_FOLD=str(fold)))


@pytest.mark.parametrize("fixture", ["g3_anderson3d", "g4_banded", "g5_anderson2d_sa",
                                     "g6_anderson2d_be", "g10_anderson2d_sm"])
def test_folded_equals_unfolded_and_reference(tmp_path, golden, fixture):
    g = golden(fixture)
    fo = _solve(tmp_path, fixture, 1)
    un = _solve(tmp_path, fixture, 0)
    for k in ("iters", "nopx", "nrorth", "nitref", "info"):
        assert int(fo[k]) == int(un[k]), k
    assert int(fo["iters"]) == int(g["iparam"][2]) and int(fo["nopx"]) == int(g["iparam"][8])
    scale = max(1.0, np.abs(g["d"]).max())
    np.testing.assert_allclose(np.sort(fo["d"]), np.sort(g["d"]), rtol=0,
                               atol=max(1e-10, 10 * float(g["tol"])) * scale)
    np.testing.assert_allclose(np.sort(fo["d"]), np.sort(un["d"]), rtol=0, atol=1e-12 * scale)
    z, zu = fo["z"], un["z"]
    assert np.abs(z.T @ z - np.eye(z.shape[1])).max() < 1e-12
    for c in range(z.shape[1]):
        s = np.sign(z[:, c] @ zu[:, c])
        assert np.abs(s * z[:, c] - zu[:, c]).max() < 1e-8, c


def test_folded_widest_basis(pkg):
    """ncv = 64: the widest folded pass (63 formed columns + the raw one) and the
    restart's T(1:k,1:k) upload over several cycles, against the reference."""
    A = M.to_scipy(*M.anderson(24, 2, 4.0, 11))
    n, nev, ncv = A.shape[0], 24, 64
    v0 = M.dlarnv_uniform(n)[0]
    want = ref.dsaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LA", 1e-10, v0=v0, mxiter=300)
    op = pkg.CSR.from_arrays(A.indptr.astype(np.int64), A.indices, A.data)
    d, z, res = pkg.eigsh(op, n, nev, ncv, "LA", 1e-10, v0=v0, mxiter=300, device=True)
    assert res["info"] == int(want["info"]) == 0
    assert res["iters"] == int(want["iparam"][2]) and res["iters"] > 1
    assert res["nopx"] == int(want["iparam"][8])
    dw = np.sort(np.asarray(want["d"]))
    np.testing.assert_allclose(np.sort(d), dw, rtol=0, atol=1e-10 * np.abs(dw).max())
    r = np.linalg.norm(A @ z - z * d, axis=0)
    assert np.all(r <= 1e-8 * np.abs(dw).max()), r


@pytest.mark.parametrize("fixture", ["n2_dnsimp_tol", "n3_convdiff_lm", "n5_convdiff_li",
                                     "n7_convdiff_real"])
def test_folded_arnoldi(tmp_path, golden, fixture):
    """dnaupd: the fold's t = H s uses the full Hessenberg records.  Same restart
    cycles and OP*x count as the unfolded engine and the reference's cycles;
    Ritz values within the fixtures' pseudospectral bound (test_gpu_ns.py)."""
    from test_gpu_ns import _mat, _ritz_ok
    g = golden(fixture)
    env0 = dict(AHIP_FOLD_NS="0")
    fo = _solve(tmp_path, fixture, 1)
    un = _solve_env(tmp_path, fixture, env0)
    for k in ("iters", "nopx", "info"):
        assert int(fo[k]) == int(un[k]), k
    assert int(fo["iters"]) == int(g["iparam"][2])
    assert abs(int(fo["nrorth"]) - int(un["nrorth"])) <= 2
    nconv = int(g["iparam"][4])
    ref = g["ritzr"][:nconv] + 1j * g["ritzi"][:nconv]
    _ritz_ok(_mat(g["spec"]), fo["d"], ref, str(g["which"]), float(g["tol"]))


def test_folded_arnoldi_forced_refinement(tmp_path, golden):
    """Every step takes the second DGKS refinement (the parked folded step's
    host path, kFinFoldCoef2 with the Hessenberg daxpy): the reference's
    cycles and OP*x count, and the forced RCI driver's."""
    fixture = "n7_convdiff_real"
    g = golden(fixture)
    fo = _solve_env(tmp_path, fixture, dict(AHIP_FORCE_DGKS2="1"), "free")
    rc = _solve_env(tmp_path, fixture, dict(AHIP_FORCE_DGKS2="1"), "rci")
    assert int(fo["nitref"]) > 0
    for k in ("iters", "nopx", "nitref", "nrorth", "info"):
        assert int(fo[k]) == int(rc[k]), k
    assert int(fo["iters"]) == int(g["iparam"][2]) and int(fo["nopx"]) == int(g["iparam"][8])
    np.testing.assert_array_equal(fo["d"], rc["d"])
