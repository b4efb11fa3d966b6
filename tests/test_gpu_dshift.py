"""GPU: the device shift-invert operator of the symmetric engine (csrc/dshift.hip:
conjugate gradients or MINRES on the real CSR operator) and dsaupd in mode 3
with it as OP (arpack_hip_dsaupd_shift).

  * the solve against SciPy's direct solve (true residual ||(A - sigma I) y - x||
    <= 1e-11 ||x||), full and symmetric storage; b = 0 gives y = 0;
  * a negative-definite shift (sigma above the spectrum) breaks CG down: the
    solve reports -1 and a mode-3 run served by it ends with info = -9999;
  * mode 3 on the reference's m2 fixture (tests/golden/m2_sym_std_si: the
    reference's dsaupd_ in mode 3 with a sparse-LU OP, EXAMPLES/SYM/dsdrv2.f's
    setting: 1-D FEM stiffness n = 400, sigma = 0, nev 4, ncv 20, tol 1e-10):
    the same restart cycles, OP*x count and converged set, eigenvalues within
    1e-9 relative;
  * eigsh(CSR, sigma=...) on a 2-D Laplacian against SciPy's eigsh(sigma=...);
  * MINRES with sigma inside the spectrum (indefinite A - sigma I): the solve
    against SciPy's direct solve, and interior eigenvalues against the exact
    spectrum (parity unpinned by a reference fixture: analytic answers).
"""
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp
import scipy.sparse.linalg as spl

from oracle import matrices as M

sys.path.insert(0, os.path.dirname(__file__))
import modes  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("method", ["cg", "minres"])
@pytest.mark.parametrize("storage", ["full", "sym"])
@pytest.mark.parametrize("sigma", [0.0, -0.5])
def test_dshift_solve(pkg, storage, sigma, method):
    m = 120
    A = pkg.CSR.laplace2d(m)
    As = M.to_scipy(*M.laplace2d(m))
    if storage == "sym":
        A.set_symmetric(True)
    n = m * m
    S = pkg.DShift(A, sigma, rtol=1e-12, maxit=2000, method=method)
    x = np.random.default_rng(3).uniform(-1, 1, n)
    y, it, rr = S.solve(x)
    assert it > 0 and rr <= 1e-12, (it, rr)
    true = np.linalg.norm(As @ y - sigma * y - x) / np.linalg.norm(x)
    assert true <= 1e-11, true
    yref = spl.spsolve((As - sigma * sp.identity(n)).tocsc(), x)
    assert np.linalg.norm(y - yref) <= 1e-9 * np.linalg.norm(yref)
    y0, it0, _ = S.solve(np.zeros(n))
    assert it0 == 0 and not y0.any()
    st = S.stats()
    assert st["solves"] == 2 and st["failures"] == 0 and st["iters"] == it


def test_dshift_negative_definite_fails_loudly(pkg):
    m = 40
    A = pkg.CSR.laplace2d(m)  # spectrum in (0, 8)
    S = pkg.DShift(A, 10.0, rtol=1e-12, maxit=500)
    y, it, rr = S.solve(np.ones(m * m))
    assert it == -1 and S.stats()["failures"] == 1
    s = pkg.SymRci(m * m, 4, 20, "LM", 1e-10, mode=3, mxiter=50)
    assert s.aupd_shift(S) == 99 and int(s.info[0]) == -9999


@pytest.mark.parametrize("method", ["cg", "minres"])
def test_dsaupd_mode3_device_solve_m2(pkg, golden, method):
    g = golden("m2_sym_std_si")
    n, sigma = int(g["n"]), float(g["sigma"])
    c = modes.StdShiftInvert(str(g["kind"]), n, sigma)
    Acsr = c.A.tocsr()
    A = pkg.CSR.from_arrays(Acsr.indptr, Acsr.indices, Acsr.data)
    S = pkg.DShift(A, sigma, rtol=1e-13, maxit=4000, method=method)
    s = pkg.SymRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), mode=3,
                   mxiter=300, v0=g["v0"])
    assert s.aupd_shift(S) == 99
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[2]) == int(g["iparam"][2])
    assert int(s.iparam[4]) == int(g["iparam"][4])
    assert int(s.iparam[8]) == int(g["nopx"])
    st = S.stats()
    assert st["solves"] == int(s.iparam[8]) and st["failures"] == 0
    d, z, nconv = s.eupd(sigma=sigma)
    dref = np.sort(g["d"])
    np.testing.assert_allclose(np.sort(d), dref, rtol=1e-9, atol=0)


def test_eigsh_shift_invert_laplace2d(pkg):
    m = 60
    A = pkg.CSR.laplace2d(m)
    As = M.to_scipy(*M.laplace2d(m))
    n = m * m
    v0 = np.random.default_rng(5).uniform(-1, 1, n)
    d, z, res = pkg.eigsh(A, n, nev=6, ncv=20, which="LM", tol=1e-12, v0=v0, sigma=0.0)
    assert res["info"] == 0 and res["nconv"] == 6
    # the square grid's spectrum is degenerate (lambda_ij = lambda_ji), where
    # ARPACK may return one copy of a double eigenvalue and the next one (SciPy
    # does here) or both copies: every Ritz value must be an exact eigenvalue
    # among the smallest, and agree with SciPy's eigsh(sigma=0) where both have it
    c = 2.0 * np.cos(np.arange(1, m + 1) * np.pi / (m + 1))
    exact = np.sort((4.0 - c[:, None] - c[None, :]).ravel())
    for x in d:
        assert np.abs(exact - x).min() <= 1e-9 * x
        assert x <= exact[7] * (1 + 1e-9)
    dref = spl.eigsh(As.tocsc(), k=6, ncv=20, sigma=0.0, which="LM", tol=1e-12, v0=v0,
                     return_eigenvectors=False)
    for x in dref:
        if x <= np.max(d):
            assert np.abs(d - x).min() <= 1e-9 * x, (x, d)
    for k in range(6):
        r = np.linalg.norm(As @ z[:, k] - d[k] * z[:, k])
        assert r <= 1e-9 * 8.0 * np.linalg.norm(z[:, k])


def test_minres_indefinite_solve(pkg):
    """sigma inside the spectrum: A - sigma I indefinite, where CG breaks down and
    MINRES converges (true residual <= 1e-10 ||x||, against SciPy's direct solve)."""
    m = 40
    A = pkg.CSR.laplace2d(m)
    As = M.to_scipy(*M.laplace2d(m))
    n = m * m
    sigma = 3.93
    x = np.random.default_rng(9).uniform(-1, 1, n)
    S = pkg.DShift(A, sigma, rtol=1e-12, maxit=20000, method="minres")
    y, it, rr = S.solve(x)
    assert it > 0 and rr <= 1e-12, (it, rr)
    Bs = (As - sigma * sp.identity(n)).tocsc()
    assert np.linalg.norm(Bs @ y - x) <= 1e-10 * np.linalg.norm(x)
    yref = spl.spsolve(Bs, x)
    assert np.linalg.norm(y - yref) <= 1e-8 * np.linalg.norm(yref)


def test_eigsh_interior_eigenvalues_minres(pkg):
    """Interior eigenvalues (nearest sigma = 3.93 of a 2-D Laplacian spectrum in
    (0, 8)) by shift-invert mode 3 with the device MINRES: every Ritz value an
    exact eigenvalue among the nearest to sigma, residuals <= 1e-9 ||A||."""
    m = 40
    A = pkg.CSR.laplace2d(m)
    As = M.to_scipy(*M.laplace2d(m))
    n = m * m
    sigma = 3.93
    v0 = np.random.default_rng(2).uniform(-1, 1, n)
    d, z, res = pkg.eigsh(A, n, nev=4, ncv=20, which="LM", tol=1e-10, v0=v0, sigma=sigma,
                          maxit=20000, solver="minres")
    assert res["info"] == 0 and res["nconv"] == 4
    c = 2.0 * np.cos(np.arange(1, m + 1) * np.pi / (m + 1))
    exact = (4.0 - c[:, None] - c[None, :]).ravel()
    near = exact[np.argsort(np.abs(exact - sigma))]
    for x in d:
        assert np.abs(exact - x).min() <= 1e-9 * abs(x)
        assert abs(x - sigma) <= abs(near[7] - sigma) * (1 + 1e-9)
    for k in range(4):
        r = np.linalg.norm(As @ z[:, k] - d[k] * z[:, k])
        assert r <= 1e-9 * 8.0 * np.linalg.norm(z[:, k])


def test_dnaupd_mode3_bicgstab_unreachable_fails_loudly(pkg, golden):
    """dndrv2's operator (the m7 fixture: 1-D convection-diffusion n = 400,
    sigma = 1) is strongly non-normal: BiCGStab takes ~3,500 iterations to
    1e-10 and stagnates near 2e-11 (measured), where the reference factors the
    tridiagonal A - sigma I directly (dgttrf/dgttrs).  A device solve that
    cannot reach its rtol is never passed on as OP: the mode-3 run ends with
    info = -9999 instead of returning eigenvalues of a perturbed operator."""
    g = golden("m7_ns_std_si")
    n, sigma = int(g["n"]), float(g["sigma"])
    c = modes.StdShiftInvert(str(g["kind"]), n, sigma)
    Acsr = c.A.tocsr()
    A = pkg.CSR.from_arrays(Acsr.indptr, Acsr.indices, Acsr.data)
    S = pkg.DShift(A, sigma, rtol=1e-12, maxit=500, method="bicgstab")
    s = pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), mode=3,
                  mxiter=300, v0=g["v0"])
    assert s.aupd_shift(S) == 99
    assert int(s.info[0]) == -9999
    assert S.stats()["failures"] == 1


def test_eigs_real_shift_invert(pkg):
    """eigs(CSR, sigma=...) -- dnaupd mode 3, device BiCGStab -- on dndrv1's 2-D
    convection-diffusion operator against SciPy's eigs(sigma=...): the
    eigenvalues nearest a shift where A - sigma I is well conditioned (the
    Krylov solve's domain; see the m7 test above for one where it is not)."""
    m, rho = 30, 10.0
    A = pkg.CSR.convdiff2d(m, rho)
    As = M.to_scipy(*M.convdiff2d(m, rho))
    n = m * m
    sigma = -100.0  # left of the spectrum (real parts ~20..3,800): A - sigma I well conditioned
    v0 = np.random.default_rng(12).uniform(-1, 1, n)
    d, z, res = pkg.eigs(A, n, nev=6, ncv=20, which="LM", tol=1e-12, v0=v0, sigma=sigma,
                         maxit=5000)
    assert res["info"] == 0 and res["nconv"] >= 6
    dref = spl.eigs(As.tocsc(), k=6, ncv=20, sigma=sigma, which="LM", tol=1e-12, v0=v0,
                    return_eigenvectors=False)
    for x in dref:
        assert np.abs(d - x).min() <= 1e-9 * np.abs(dref).max(), (x, d)
    an = abs(As).sum(axis=0).max()
    for k in range(len(d)):
        r = np.linalg.norm(As @ z[:, k] - d[k] * z[:, k])
        assert r <= 1e-9 * an * np.linalg.norm(z[:, k])


@pytest.mark.parametrize("n", [1, 2, 3, 17, 4099, 1_000_003])
def test_tridiag_direct_solve(pkg, n):
    """DShift method "tridiag" (csrc/dtri.hip): dgttrf on the host, the two
    triangular solves as device scans of affine maps -- against SciPy's
    (LAPACK) dgttrs on a random nonsymmetric tridiagonal that pivots, at sizes
    that put the segment and block boundaries everywhere (1 .. 10^6 rows)."""
    import scipy.linalg.lapack as lapack
    rng = np.random.default_rng(n)
    dl, d, du = rng.standard_normal(n - 1), rng.standard_normal(n) + 0.5, rng.standard_normal(n - 1)
    sigma = 0.25
    A = sp.diags([dl, d, du], [-1, 0, 1], shape=(n, n), format="csr")
    A.sort_indices()
    Ad = pkg.CSR.from_arrays(A.indptr, A.indices, A.data)
    S = pkg.DShift(Ad, sigma, method="tridiag")
    b = rng.standard_normal(n)
    y, it, rr = S.solve(b)
    assert it == 1
    if n >= 3:
        f = lapack.dgttrf(dl, d - sigma, du)
        xr, info = lapack.dgttrs(*f[:5], b)
        assert info == 0
    else:
        xr = np.linalg.solve((A - sigma * sp.identity(n)).toarray(), b)
    np.testing.assert_allclose(y, xr, rtol=0, atol=1e-10 * np.abs(xr).max())
    r = (A - sigma * sp.identity(n)) @ y - b
    assert np.linalg.norm(r) <= 1e-9 * np.linalg.norm(b) * max(1.0, np.abs(xr).max())


def test_tridiag_refuses_wider_operator(pkg):
    """method "tridiag" needs a tridiagonal A: anything wider is refused."""
    A = pkg.CSR.laplace2d(10)
    with pytest.raises(ValueError):
        pkg.DShift(A, 0.0, method="tridiag")


def test_dnaupd_mode3_tridiag_m7(pkg, golden):
    """dndrv2 as the reference runs it (the m7 fixture: A - sigma I factored
    directly, EXAMPLES/NONSYM/dndrv2.f:197-258) with the device's direct
    tridiagonal solve as OP: the reference's info, nconv, restart cycles and
    OP*x, and every eigenvalue of its dneupd within 1e-9 (relative to the
    largest) of one of ours -- the case BiCGStab cannot serve (above)."""
    g = golden("m7_ns_std_si")
    n, sigma = int(g["n"]), float(g["sigma"])
    c = modes.StdShiftInvert(str(g["kind"]), n, sigma)
    Acsr = c.A.tocsr()
    Acsr.sort_indices()
    A = pkg.CSR.from_arrays(Acsr.indptr, Acsr.indices, Acsr.data)
    S = pkg.DShift(A, sigma, method="tridiag")
    s = pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), mode=3,
                  mxiter=300, v0=g["v0"], device=True)
    assert s.aupd_shift(S) == 99
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[4]) == int(g["iparam"][4])
    assert int(s.iparam[2]) == int(g["iparam"][2]), (int(s.iparam[2]), int(g["iparam"][2]))
    assert int(s.iparam[8]) == int(g["iparam"][8])
    dr, di, z, nconv = s.eupd(sigmar=sigma)
    lam, ref = dr[:nconv] + 1j * di[:nconv], g["dr"] + 1j * g["di"]
    for x in ref:
        assert np.abs(lam - x).min() <= 1e-9 * np.abs(ref).max(), (x, lam)
