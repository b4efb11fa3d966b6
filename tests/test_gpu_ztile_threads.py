"""The complex tiles' workgroup size (AHIP_ZTILE_T = 256 / 512 / 1,024
threads, zsplit.hip k_ztile / k_ztile_det) and the entries a lane keeps in
flight (AHIP_ZTILE_U; 6 by default at 1,024 threads) change how many waves
share a tile's LDS row sums and in what order they add, not what is summed: the deterministic form's exact
fixed-point sums are bitwise the same at every size, and the default form's
LDS-atomic sums agree to rounding with each other and with SciPy.  The size is
read once a process, so each runs in a subprocess."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _run(tmp_path, threads, unroll=None):
    out = tmp_path / f"t{threads}_u{unroll}.npz"
    env = dict(os.environ, AHIP_ZTILE_T=str(threads))
    env.pop("AHIP_ZTILE_U", None)
    if unroll:
        env["AHIP_ZTILE_U"] = str(unroll)
    r = subprocess.run([sys.executable, os.path.join(HERE, "ztile_worker.py"), str(out)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return dict(np.load(out))


def test_tile_threads_same_products(tmp_path):
    import scipy.sparse as sp
    runs = {(t, None): _run(tmp_path, t) for t in (256, 512, 1024)}
    for u in (4, 8):  # 1,024 threads: four entries a lane, and eight (k_ztile_w8)
        runs[(1024, u)] = _run(tmp_path, 1024, u)
    base = runs[(256, None)]
    n = base["x"].size
    S = sp.csr_matrix((base["val"], base["col"], base["rp"]), shape=(n, n))
    ref = S @ base["x"]
    scale = 64 * np.finfo(float).eps * (abs(S) @ np.abs(base["x"]))
    for t, r in runs.items():
        np.testing.assert_array_equal(r["x"], base["x"])
        np.testing.assert_array_equal(r["yd"].view(np.int64), base["yd"].view(np.int64))
        assert np.all(np.abs(r["y"] - ref) <= 2 * scale + 1e-300), t
        assert np.all(np.abs(r["y"] - base["y"]) <= 2 * scale + 1e-300), t
