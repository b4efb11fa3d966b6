"""GPU: Krylov bases wider than the kernels' fast-path tiles, against the
reference run in-process (oracle/_ref), same operator and start vector.

The reference accepts any ncv <= n (SRC/dsaupd.f:511, SRC/dnaupd.f:442,
SRC/znaupd.f:478).  The engine's fast paths hold fixed tiles: the CGS/DGKS
finalize stages ncv + 2 sums (now dynamic LDS), V*Q keeps a row of <= 64
coefficients in registers, the eupd products <= 128 (complex <= 64), and the
complex update stages 256 coefficients in LDS.  These cases take every one of
them past its tile, so the generic kernels (per-thread scratch columns) and the
strided finalize loops run:

* dsaupd ncv = 300 (finalize m = 302 > 256 slots; V*Q kplusp = 300 > 64;
  dseupd V*Q with k = 300 > 128), host RCI and the free-running device loop;
* dnaupd ncv = 280 (H columns recorded for j up to 280; dnapps V*Q kplusp = 280;
  dneupd gemm k = 280);
* znaupd ncv = 270 (complex update with j up to 270 > 256; znapps / zneupd
  zgemm k = 270 > 64).

Ritz values within 1e-9 relative of the reference's, restart cycles equal,
Ritz-vector residuals <= 1e-8 |lambda|max.  The ncv > 8000 rejection (info = -3)
is the CPU test tests/test_arg_errors.py::test_ncv_above_engine_limit.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import matrices as M
from oracle import ref

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not ref.available(), reason="oracle/_ref")]


def _close(got, exp, rel=1e-9):
    scale = max(1.0, np.abs(exp).max())
    assert np.all(np.abs(got - exp) <= rel * scale), (got, exp)


@pytest.mark.parametrize("device", [False, True])
def test_dsaupd_ncv300(pkg, device):
    A = M.to_scipy(*M.anderson(40, 2, 4.0, 7))  # n = 1600
    n, nev, ncv = A.shape[0], 20, 300
    v0 = M.dlarnv_uniform(n)[0]
    want = ref.dsaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LA", 1e-10, v0=v0, mxiter=300)
    op = pkg.CSR.from_arrays(A.indptr.astype(np.int64), A.indices, A.data) if device else (
        lambda x: A @ x)
    d, z, res = pkg.eigsh(op, n, nev, ncv, "LA", 1e-10, v0=v0, mxiter=300, device=device)
    assert res["info"] == want["info"]
    assert res["nconv"] == want["nconv"]
    assert res["iters"] == int(want["iparam"][2]), (res, want["iparam"])
    _close(np.sort(d), np.sort(want["d"]))
    r = np.linalg.norm(A @ z - z * d, axis=0)
    assert np.all(r <= 1e-8 * np.abs(d).max()), r


def _ns_op(n, seed):
    # well-conditioned nonsymmetric: spread real diagonal + small random coupling
    rng = np.random.default_rng(seed)
    B = sp.random(n, n, density=8.0 / n, random_state=rng, format="csr")
    B.data = np.round(B.data * 64.0) / 256.0
    return (B + sp.diags(np.arange(1.0, n + 1.0))).tocsr()


def test_dnaupd_ncv280(pkg):
    A = _ns_op(3000, 3)  # 3 restart cycles at ncv = 280
    n, nev, ncv = A.shape[0], 12, 280
    v0 = M.dlarnv_uniform(n)[0]
    want = ref.dnaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LM", 1e-10, v0=v0, mxiter=300,
                            rvec=False)
    s = pkg.NsRci(n, nev, ncv, "LM", 1e-10, mxiter=300, v0=v0)
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        elif ido == 99:
            break
        else:
            raise AssertionError(ido)
    assert int(s.info[0]) == want["info"]
    assert int(s.iparam[2]) == int(want["iparam"][2])
    dr, di, z, nconv = s.eupd(rvec=True)
    assert nconv == want["nconv"]
    got = np.sort_complex(dr[:nconv] + 1j * di[:nconv])
    exp = np.sort_complex(want["dr"] + 1j * want["di"])
    _close(got, exp)
    # real spectrum here (diagonal-dominant upper/lower mix): Z columns are eigenvectors
    assert np.all(di[:nconv] == 0.0)
    Z = np.asarray(z).reshape(nev + 1, n)[:nconv].T
    r = np.linalg.norm(A @ Z - Z * dr[:nconv], axis=0)
    assert np.all(r <= 1e-8 * np.abs(dr[:nconv]).max()), r


def test_znaupd_ncv270(pkg):
    rp, col, val = M.zrandom(3000, 20, 5, 100.0)  # 4 restart cycles at ncv = 270
    A = sp.csr_matrix((val, col, rp), shape=(3000, 3000))
    n, nev, ncv = 3000, 8, 270
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)
    want = ref.znaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LM", 1e-10, v0=v0, rvec=False)
    s = pkg.ZRci(n, nev, ncv, "LM", 1e-10, v0=v0)
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        elif ido == 99:
            break
        else:
            raise AssertionError(ido)
    assert int(s.info[0]) == want["info"]
    assert int(s.iparam[2]) == int(want["iparam"][2])
    d, z, nconv = s.eupd(rvec=True)
    assert nconv == want["nconv"]
    got, exp = np.sort_complex(d[:nconv]), np.sort_complex(want["d"])
    _close(got, exp)
    Z = z[:, :nconv]
    r = np.linalg.norm(A @ Z - Z * d[:nconv], axis=0)
    assert np.all(r <= 1e-8 * np.abs(d[:nconv]).max()), r
