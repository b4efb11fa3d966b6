"""GPU parity at the north star's full size (BASELINE: dsaupd on the NS operator,
n = 1e7, ~51 nnz/row, LA, nev = 10, ncv = 30) -- the bench's time-to-converge
case, tol = 1e-6, v0 = dlarnv(1,3,5,7).

The reference (oracle/_ref, run in a subprocess by oracle/fullsize_ref.py with
16 BLAS/OpenMP threads, ~40 s) and the engine (device CSR free run, full and
symmetric storage) solve the same operator from the same start vector:
  * same info, nconv, restart cycles iparam(3) and OP*x count;
  * Ritz values |d - d_ref| <= 1e-10 * max(1, |d_ref|)  (SURVEY.md §8c);
  * the engine's Ritz vectors: ||A z - d z|| <= 10 * tol * |d| (ARPACK's own
    acceptance, bounds(i) <= tol * |ritz(i)|), evaluated with the device SpMV.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle.cpu_baseline import dlarnv_fast

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, NEV, NCV, TOL = 10_000_000, 10, 30, 1e-6


@pytest.fixture(scope="module")
def reference(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("fullsize") / "ref.npz")
    threads = min(16, len(os.sched_getaffinity(0)))
    r = subprocess.run([sys.executable, "-m", "oracle.fullsize_ref", "--n", str(N), "--threads",
                        str(threads), "--out", out], cwd=ROOT, capture_output=True, text=True,
                       timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    print(r.stdout.strip())
    return dict(np.load(out, allow_pickle=False))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("storage", ["full", "sym"])
def test_north_star_full_size(pkg, reference, storage):
    ref = reference
    assert int(ref["info"]) == 0 and int(ref["nconv"]) == NEV
    A = pkg.CSR.banded_sym(N)
    if storage == "sym":
        A.set_symmetric(True)
    s = pkg.SymRci(N, NEV, NCV, "LA", TOL, mxiter=300, v0=dlarnv_fast(N), device=True)
    s.aupd_csr(A)
    assert int(s.info[0]) == 0 and int(s.iparam[4]) == NEV
    assert int(s.iparam[2]) == int(ref["iparam"][2])
    assert int(s.iparam[8]) == int(ref["nopx"])
    dv, zb, nconv = s.eupd(rvec=True)
    assert nconv == NEV
    d = np.sort(dv)
    assert np.all(np.abs(d - ref["d"]) <= 1e-10 * np.maximum(1.0, np.abs(ref["d"]))), \
        np.abs(d - ref["d"]).max()
    # Ritz vectors: residuals with the device SpMV
    y = pkg.DeviceBuffer(N)
    for k in range(nconv):
        A.matvec_device(zb.at(k * N), y)
        zk = zb.numpy(k * N, N)
        r = np.linalg.norm(y.numpy() - dv[k] * zk)
        assert r <= 10 * TOL * abs(dv[k]), (k, r, dv[k])
