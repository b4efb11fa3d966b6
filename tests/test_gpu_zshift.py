"""GPU: the device shift-invert operator (csrc/zsolve.hip, BiCGStab on the complex
CSR operator) and znaupd in mode 3 with it as OP (arpack_hip_znaupd_zshift).

  * the solve against SciPy's product (true residual ||(A - sigma I) y - x|| /
    ||x|| <= 1e-11) and against the host restatement oracle/krylov.py (same
    iteration, iterates to 1e-10 relative, iteration counts within one), on the
    wave-per-row SpMV (n = 2000) and the XCD-split SpMV (n = 3e5);
  * b = 0 gives y = 0 in zero iterations; a solve that cannot reach rtol in
    maxit reports -1 and is counted as a failure;
  * mode 3 free run on the reference's z3 fixture (tests/golden/z3_zrandom_si:
    the reference's znaupd_ in mode 3 with a sparse-LU OP, sigma = 0, nev 6,
    ncv 20, tol 1e-10): the same converged set, eigenvalues within
    max(1e-9, 10 tol) relative, Ritz residuals within 10x the reference's.
The full-size config-5 run (n = 5e5) is in tests/test_gpu_fullsize.py.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import matrices as M
from oracle.krylov import bicgstab

pytestmark = pytest.mark.gpu


def _op(rp, col, val):
    n = len(rp) - 1
    return sp.csr_matrix((val, col, rp), shape=(n, n))


@pytest.mark.parametrize("n,per,seed,sigma", [(2000, 20, 5, 0j), (2000, 20, 5, 0.5 + 0.25j),
                                              (300000, 64, 7, 0j), (300000, 64, 7, 3.0 - 2.0j)])
def test_zshift_solve(pkg, n, per, seed, sigma):
    Z = pkg.ZCSR.random(n, per, seed, 100.0)
    A = _op(*Z.download())
    S = pkg.ZShift(Z, sigma, rtol=1e-12, maxit=100)
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    y, it, rr = S.solve(x)
    assert it > 0 and rr <= 1e-12, (it, rr)
    true = np.linalg.norm(A @ y - sigma * y - x) / np.linalg.norm(x)
    assert true <= 1e-11, true
    yh, ith, rrh, ok = bicgstab(lambda v: A @ v, x, sigma, 1e-12, 100)
    assert ok and abs(ith - it) <= 1, (it, ith)
    assert np.linalg.norm(y - yh) <= 1e-10 * np.linalg.norm(yh)
    st = S.stats()
    assert st["solves"] == 1 and st["iters"] == it and st["failures"] == 0
    assert st["ms"] > 0 and st["bytes_per_iter"] > 20 * Z.nnz


def test_zshift_zero_rhs_and_failure(pkg):
    Z = pkg.ZCSR.random(2000, 20, 5, 100.0)
    S = pkg.ZShift(Z, 0j, rtol=1e-12, maxit=50)
    y, it, rr = S.solve(np.zeros(2000, complex))
    assert it == 0 and not y.any()
    F = pkg.ZShift(Z, 0j, rtol=1e-30, maxit=2)  # unreachable tolerance
    x = np.ones(2000, complex)
    y, it, rr = F.solve(x)
    assert it == -1 and rr > 0
    assert F.stats()["failures"] == 1
    # the solver is reusable after a failure
    G = pkg.ZShift(Z, 0j, rtol=1e-12, maxit=50)
    y, it, rr = G.solve(x)
    assert it > 0 and rr <= 1e-12


def _resid(A, z, d):
    anorm = abs(A).sum(axis=0).max()
    return max(np.linalg.norm(A @ z[:, k] - d[k] * z[:, k]) / (anorm * np.linalg.norm(z[:, k]))
               for k in range(len(d)))


def test_znaupd_mode3_device_solve_z3(pkg, golden):
    g = golden("z3_zrandom_si")
    spec = g["spec"]
    n, per, seed, dsh = int(spec[1]), int(spec[2]), int(spec[3]), float(spec[4])
    Z = pkg.ZCSR.random(n, per, seed, dsh)
    A = _op(*M.zrandom(n, per, seed, dsh))
    sigma = complex(g["sigma"])
    S = pkg.ZShift(Z, sigma, rtol=1e-13, maxit=200)
    s = pkg.ZRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), mode=3,
                 mxiter=int(g["mxiter"]), v0=g["v0"])
    assert s.aupd_zshift(S) == 99
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[4]) == int(g["iparam"][4])
    st = S.stats()
    assert st["solves"] == int(s.iparam[8]) and st["failures"] == 0
    print("OP*x %d (reference %d), restart cycles %d (reference %d), %.1f BiCGStab iterations a solve"
          % (s.iparam[8], g["iparam"][8], s.iparam[2], g["iparam"][2], st["iters"] / st["solves"]))
    d, z, nc = s.eupd(sigma=sigma)
    dref = g["d"]
    tol = max(1e-9, 10 * float(g["tol"])) * np.abs(dref).max()
    for x in dref:
        assert np.abs(d - x).min() <= tol, (x, d)
    ours, theirs = _resid(A, z, d), _resid(A, g["z"], dref)
    assert ours <= max(10 * theirs, 1e-12), (ours, theirs)


def test_znaupd_mode3_argument_checks(pkg):
    Z = pkg.ZCSR.random(2000, 20, 5, 100.0)
    S = pkg.ZShift(Z, 0j)
    s = pkg.ZRci(2000, 6, 20, "LM", 1e-10, mode=1)  # the device solve serves mode 3 only
    assert s.aupd_zshift(S) == 99 and int(s.info[0]) == -11
    s = pkg.ZRci(1999, 6, 20, "LM", 1e-10, mode=3)  # n must be the operator's
    assert s.aupd_zshift(S) == 99 and int(s.info[0]) == -11


def test_zshift_singular_shift_fails_loudly(pkg):
    """sigma on an eigenvalue: A - sigma I is singular, BiCGStab cannot reach
    rtol -- the solve reports -1 (a counted failure, never a silent result) and
    a mode-3 run served by it ends with info = -9999."""
    rp, col, val = M.zdiag_icb(1000)  # diag (k+1)(1+i)
    Z = pkg.ZCSR.from_arrays(rp, col, val)
    S = pkg.ZShift(Z, 5 * (1 + 1j), rtol=1e-12, maxit=30)
    x = np.random.default_rng(1).standard_normal(1000) + 0j
    _, it, rr = S.solve(x)
    assert it == -1
    assert S.stats()["failures"] == 1
    s = pkg.ZRci(1000, 4, 12, "LM", 1e-8, mode=3, mxiter=50)
    assert s.aupd_zshift(S) == 99
    assert int(s.info[0]) == -9999


def _tridiag(n, rho=10.0, seed=None):
    """zndrv2's operator (1/h^2 scaling) or, with a seed, a random complex
    tridiagonal that pivots."""
    if seed is None:
        h = 1.0 / (n + 1)
        s = rho / 2.0
        lo = np.full(n - 1, -1.0 / h**2 - s / h, np.complex128)
        di = np.full(n, 2.0 / h**2, np.complex128)
        up = np.full(n - 1, -1.0 / h**2 + s / h, np.complex128)
    else:
        rng = np.random.default_rng(seed)
        c = lambda k: rng.standard_normal(k) + 1j * rng.standard_normal(k)  # noqa: E731
        lo, di, up = c(n - 1), c(n), c(n - 1)
    return sp.diags([lo, di, up], [-1, 0, 1], shape=(n, n), format="csr", dtype=np.complex128)


@pytest.mark.parametrize("n,seed,sigma", [(1, 3, 0j), (2, 3, 0j), (3, 3, 0.5j), (17, 3, 0j),
                                          (4099, 5, 1 - 1j), (100, None, 0j),
                                          (1000003, 7, 0.25 + 0.5j)])
def test_ztridiag_direct_solve(pkg, n, seed, sigma):
    """ZShift method 1 (zgttrf on the host, the triangular solves as device
    scans, csrc/ztri.hip) against SciPy's sparse LU of A - sigma I: the
    relative true residual and the solution to LU's rounding."""
    import scipy.sparse.linalg as spl
    A = _tridiag(n, seed=seed)
    A.sort_indices()
    Z = pkg.ZCSR.from_arrays(A.indptr, A.indices, A.data)
    S = pkg.ZShift(Z, sigma, method="tridiag")
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    y, it, rr = S.solve(x)
    assert it == 0 and rr == 0.0
    C = (A - sigma * sp.identity(n, format="csr", dtype=np.complex128)).tocsc()
    yr = spl.splu(C).solve(x) if n > 1 else x / C.toarray()[0, 0]
    assert np.linalg.norm(C @ y - x) <= 1e-10 * np.linalg.norm(x) * max(1.0, np.abs(C).max())
    assert np.abs(y - yr).max() <= 1e-9 * np.abs(yr).max()


def test_ztridiag_refuses_wider_operator(pkg):
    Z = pkg.ZCSR.random(2000, 20, 5, 100.0)
    with pytest.raises(ValueError):
        pkg.ZShift(Z, 0j, method="tridiag")


@pytest.mark.parametrize("name", ["z8_zndrv2_si", "z9_zndrv2_si_shift"])
def test_znaupd_mode3_tridiag_zndrv2(pkg, golden, name):
    """EXAMPLES/COMPLEX/zndrv2.f's shift-invert run, free on the device with
    the direct tridiagonal solve (the driver's zgttrf / zgttrs): the
    reference's info, nconv, restart cycles and OP*x count, eigenvalues within
    1e-9 of the largest."""
    g = golden(name)
    n = int(g["spec"][1])
    A = _tridiag(n, rho=float(g["spec"][2]))
    A.sort_indices()
    Z = pkg.ZCSR.from_arrays(A.indptr, A.indices, A.data)
    sigma = complex(g["sigma"])
    S = pkg.ZShift(Z, sigma, method="tridiag")
    s = pkg.ZRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), mode=3,
                 mxiter=int(g["mxiter"]), v0=g["v0"])
    assert s.aupd_zshift(S) == 99
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[4]) == int(g["iparam"][4])
    assert int(s.iparam[2]) == int(g["iparam"][2]), (int(s.iparam[2]), int(g["iparam"][2]))
    assert int(s.iparam[8]) == int(g["iparam"][8])
    assert S.stats()["solves"] == int(s.iparam[8])
    d, z, nc = s.eupd(sigma=sigma)
    dref = g["d"]
    for x in dref:
        assert np.abs(d - x).min() <= 1e-9 * np.abs(dref).max(), (x, d)
