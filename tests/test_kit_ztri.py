"""CPU: the complex tridiagonal direct solve's host half (csrc/ztri.hip:
zgttrf and zgttrs restated, pivoting by |re| + |im| as LAPACK's zgttrf does;
arpack_hip_kit_zgttrf / _zgttrs) against the image's LAPACK through SciPy, on
random complex tridiagonals that do and do not pivot, and on the operator of
the reference's zndrv2 (EXAMPLES/COMPLEX/zndrv2.f: the 1-D convection-diffusion
with 1/h^2 scaling, rho = 10) shifted by a complex sigma.  The device solve
evaluates the same triangular recurrences as scans (tests/test_gpu_zshift.py)."""
import ctypes as C

import numpy as np
import pytest
import scipy.linalg.lapack as lapack

PD = C.POINTER(C.c_double)
PI = C.POINTER(C.c_int)


def _kit(pkg):
    L = pkg.lib()
    L.arpack_hip_kit_zgttrf.argtypes = [C.c_int64, PD, PD, PD, PD, PI]
    L.arpack_hip_kit_zgttrs.argtypes = [C.c_int64, PD, PD, PD, PD, PI, PD]
    return L


def _pd(a):
    return a.ctypes.data_as(PD)


def _factor(L, dl, d, du):
    n = len(d)
    m = max(n, 1)
    fdl, fd, fdu, fu2 = (np.zeros(m, np.complex128) for _ in range(4))
    fdl[:n - 1], fd[:n], fdu[:n - 1] = dl, d, du
    ipiv = np.zeros(m, np.int32)
    info = L.arpack_hip_kit_zgttrf(n, _pd(fdl), _pd(fd), _pd(fdu), _pd(fu2), ipiv.ctypes.data_as(PI))
    return info, fdl, fd, fdu, fu2, ipiv


def zndrv2(n, rho=10.0, sigma=0j):
    h = 1.0 / (n + 1)
    s = rho / 2.0
    return (np.full(n - 1, -1.0 / h**2 - s / h, np.complex128),
            np.full(n, 2.0 / h**2, np.complex128) - sigma,
            np.full(n - 1, -1.0 / h**2 + s / h, np.complex128))


def _cases():
    rng = np.random.default_rng(11)
    c = lambda *s: rng.standard_normal(s) + 1j * rng.standard_normal(s)  # noqa: E731
    out = []
    for n in (3, 5, 64, 1000):
        out.append(("random", c(n - 1), c(n), c(n - 1)))
        out.append(("dominant", 0.5 * c(n - 1), 4.0 + c(n) * 0.2, 0.5 * c(n - 1)))
    out.append(("zndrv2", *zndrv2(100)))
    out.append(("zndrv2_shift", *zndrv2(100, sigma=5000 + 2000j)))
    return out


@pytest.mark.parametrize("case", range(10))
def test_zgttrf_zgttrs_match_lapack(pkg, case):
    name, dl, d, du = _cases()[case]
    L = _kit(pkg)
    n = len(d)
    info, fdl, fd, fdu, fu2, ipiv = _factor(L, dl, d, du)
    rdl, rd, rdu, rdu2, ripiv, rinfo = lapack.zgttrf(dl, d, du)
    assert info == rinfo == 0
    np.testing.assert_array_equal(ipiv[:n], ripiv - 1)  # LAPACK's pivots are 1-based
    scale = np.abs(d).max() + 1.0
    for ours, ref in ((fdl[:n - 1], rdl), (fd[:n], rd), (fdu[:n - 1], rdu),
                      (fu2[:max(n - 2, 0)], rdu2[:max(n - 2, 0)])):
        np.testing.assert_allclose(ours, ref, rtol=1e-13, atol=1e-13 * scale)
    rng = np.random.default_rng(case)
    b = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    x = b.copy()
    L.arpack_hip_kit_zgttrs(n, _pd(fdl), _pd(fd), _pd(fdu), _pd(fu2), ipiv.ctypes.data_as(PI), _pd(x))
    xr, rinfo2 = lapack.zgttrs(rdl, rd, rdu, rdu2, ripiv, b)
    assert rinfo2 == 0
    np.testing.assert_allclose(x, xr, rtol=1e-11, atol=1e-11 * np.abs(xr).max())


def test_zsingular_reported(pkg):
    L = _kit(pkg)
    z = np.zeros(2, np.complex128)
    info, *_ = _factor(L, z, np.array([1.0, 0.0, 2.0j]), z)
    assert info == 2
