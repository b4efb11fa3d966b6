"""CPU: the tridiagonal direct solve's host half (csrc/dtri.hip: dgttrf and
dgttrs restated, arpack_hip_kit_dgttrf / _dgttrs) against the image's LAPACK
through SciPy, on random tridiagonals that do and do not pivot, and on the
operator of the reference's dndrv2 (the m7 fixture's A - sigma I).  The device
solve evaluates the same triangular recurrences as scans
(tests/test_gpu_dshift.py)."""
import ctypes as C

import numpy as np
import pytest
import scipy.linalg.lapack as lapack

PD = C.POINTER(C.c_double)


def _kit(pkg):
    L = pkg.lib()
    L.arpack_hip_kit_dgttrf.argtypes = [C.c_int64, PD, PD, PD, PD, C.POINTER(C.c_int)]
    L.arpack_hip_kit_dgttrs.argtypes = [C.c_int64, PD, PD, PD, PD, C.POINTER(C.c_int), PD]
    return L


def _factor(L, dl, d, du):
    n = len(d)
    dl2, d2, du2_ = (np.zeros(max(n, 1)) for _ in range(3))
    dl2[:n - 1], d2[:n], du2_[:n - 1] = dl, d, du
    u2 = np.zeros(max(n, 1))
    ipiv = np.zeros(max(n, 1), np.int32)
    pd = lambda a: a.ctypes.data_as(PD)  # noqa: E731
    info = L.arpack_hip_kit_dgttrf(n, pd(dl2), pd(d2), pd(du2_), pd(u2),
                                   ipiv.ctypes.data_as(C.POINTER(C.c_int)))
    return info, dl2, d2, du2_, u2, ipiv


def _cases():
    rng = np.random.default_rng(7)
    out = []
    for n in (3, 5, 64, 1000):
        out.append(("random", rng.standard_normal(n - 1), rng.standard_normal(n),
                    rng.standard_normal(n - 1)))
        # diagonally dominant: no interchange
        out.append(("dominant", rng.uniform(-1, 1, n - 1), 4.0 + rng.uniform(0, 1, n),
                    rng.uniform(-1, 1, n - 1)))
    # dndrv2's operator (1-D convection-diffusion, rho = 10, n = 400) - sigma I, sigma = 1
    n, rho = 400, 10.0
    h = 1.0 / (n + 1)
    s = rho / 2.0
    out.append(("dndrv2", np.full(n - 1, -1.0 / h - s), np.full(n, 2.0 / h - 1.0),
                np.full(n - 1, -1.0 / h + s)))
    return out


@pytest.mark.parametrize("case", range(9))
def test_dgttrf_dgttrs_match_lapack(pkg, case):
    name, dl, d, du = _cases()[case]
    L = _kit(pkg)
    n = len(d)
    info, fdl, fd, fdu, fdu2, ipiv = _factor(L, dl, d, du)
    rdl, rd, rdu, rdu2, ripiv, rinfo = lapack.dgttrf(dl, d, du)
    assert info == rinfo == 0
    np.testing.assert_array_equal(ipiv[:n], ripiv - 1)  # LAPACK's pivots are 1-based
    scale = np.abs(d).max() + 1.0
    for ours, ref in ((fdl[:n - 1], rdl), (fd[:n], rd), (fdu[:n - 1], rdu), (fu := fdu2[:max(n - 2, 0)],
                                                                               rdu2[:max(n - 2, 0)])):
        np.testing.assert_allclose(ours, ref, rtol=1e-13, atol=1e-13 * scale)
    b = np.random.default_rng(case).standard_normal(n)
    x = b.copy()
    L.arpack_hip_kit_dgttrs(n, fdl.ctypes.data_as(PD), fd.ctypes.data_as(PD), fdu.ctypes.data_as(PD),
                            fdu2.ctypes.data_as(PD), ipiv.ctypes.data_as(C.POINTER(C.c_int)),
                            x.ctypes.data_as(PD))
    xr, rinfo2 = lapack.dgttrs(rdl, rd, rdu, rdu2, ripiv, b)
    assert rinfo2 == 0
    np.testing.assert_allclose(x, xr, rtol=1e-11, atol=1e-11 * np.abs(xr).max())
    A = np.diag(d) + np.diag(dl, -1) + np.diag(du, 1) if n > 1 else np.diag(d)
    assert np.linalg.norm(A @ x - b) <= 1e-10 * np.linalg.norm(b) * max(1.0, np.linalg.cond(A) * 1e-4)


@pytest.mark.parametrize("n", [1, 2])
def test_tiny_systems(pkg, n):
    """n = 1 and 2 (SciPy's wrapper wants n >= 3): against numpy's solve."""
    L = _kit(pkg)
    rng = np.random.default_rng(n)
    dl, d, du = rng.standard_normal(n - 1), rng.standard_normal(n) + 3.0, rng.standard_normal(n - 1)
    info, fdl, fd, fdu, fdu2, ipiv = _factor(L, dl, d, du)
    assert info == 0
    b = rng.standard_normal(n)
    x = b.copy()
    L.arpack_hip_kit_dgttrs(n, fdl.ctypes.data_as(PD), fd.ctypes.data_as(PD), fdu.ctypes.data_as(PD),
                            fdu2.ctypes.data_as(PD), ipiv.ctypes.data_as(C.POINTER(C.c_int)),
                            x.ctypes.data_as(PD))
    A = np.diag(d) + (np.diag(dl, -1) + np.diag(du, 1) if n > 1 else 0)
    np.testing.assert_allclose(x, np.linalg.solve(A, b), rtol=1e-13)


def test_singular_reported(pkg):
    L = _kit(pkg)
    info, *_ = _factor(L, np.array([0.0, 0.0]), np.array([1.0, 0.0, 2.0]), np.array([0.0, 0.0]))
    assert info == 2
