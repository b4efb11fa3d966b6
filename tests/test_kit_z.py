"""CPU: the complex host kit (zdense.cpp) against the REAL reference's internal
routines (oracle/_ref: SRC/zsortc.f, zngets.f, zneigh.f, znapps.f) and the
image's LAPACK (zlahqr, ztrevc, ztrsen).  Complex arithmetic in the reference
goes through BLAS (zgemv/zrot/zscal kernels) and compiler complex division, so
these are compared to rounding level rather than bit for bit."""
import ctypes as C
import glob
import os

import numpy as np
import pytest

from oracle import ref

needs_ref = pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built")
pz = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
pi = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))  # noqa: E731
ri = lambda v: C.byref(C.c_int(v))  # noqa: E731


def _blas():
    import scipy
    p = glob.glob(os.path.join(os.path.dirname(scipy.__file__), "..", "scipy.libs",
                               "libscipy_openblas*.so"))[0]
    return C.CDLL(p)


def _hess(n, seed):
    rng = np.random.default_rng(seed)
    h = np.triu(rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)), -1)
    return np.asfortranarray(h)


def _schur(pkg, h):
    n = h.shape[0]
    t, z = h.copy(order="F"), np.asfortranarray(np.eye(n, dtype=complex))
    w = np.zeros(n, complex)
    assert pkg.lib().arpack_hip_kit_zlahqr(n, pz(t), n, pz(w), pz(z), n) == 0
    return t, z, w


@pytest.mark.parametrize("n,seed", [(5, 0), (20, 1), (40, 2)])
def test_zlahqr_matches_lapack(pkg, n, seed):
    B = _blas()
    h = _hess(n, seed)
    t1, z1 = h.copy(order="F"), np.asfortranarray(np.eye(n, dtype=complex))
    w1 = np.zeros(n, complex)
    info = C.c_int()
    one = C.c_int(1)
    B.scipy_zlahqr_(C.byref(one), C.byref(one), ri(n), ri(1), ri(n), pz(t1), ri(n), pz(w1), ri(1),
                    ri(n), pz(z1), ri(n), C.byref(info))
    t2, z2, w2 = _schur(pkg, h)
    assert info.value == 0
    np.testing.assert_allclose(w2, w1, rtol=0, atol=1e-12 * np.abs(w1).max())
    # the Schur form is unique up to a diagonal unitary D (T -> D'TD, Z -> ZD):
    # compare the D-invariant |T|, |Z| and check Z T Z^H = H, Z unitary
    np.testing.assert_allclose(np.abs(t2), np.abs(t1), rtol=0, atol=1e-11 * np.abs(t1).max())
    np.testing.assert_allclose(np.abs(z2), np.abs(z1), rtol=0, atol=1e-11)
    assert np.abs(np.tril(t2, -1)).max() == 0.0
    np.testing.assert_allclose(z2 @ t2 @ z2.conj().T, h, rtol=0, atol=1e-12 * n * np.abs(h).max())
    np.testing.assert_allclose(z2.conj().T @ z2, np.eye(n), rtol=0, atol=1e-13 * n)


@pytest.mark.parametrize("n,seed", [(6, 3), (30, 4)])
def test_ztrevc_matches_lapack(pkg, n, seed):
    B = _blas()
    t, z, w = _schur(pkg, _hess(n, seed))
    for howmny in ("A", "B"):
        vr1, vr2 = z.copy(order="F"), z.copy(order="F")
        t1, t2 = t.copy(order="F"), t.copy(order="F")
        sel = np.zeros(n, np.int32)
        m, info = C.c_int(), C.c_int()
        B.scipy_ztrevc_(C.c_char_p(b"R"), C.c_char_p(howmny.encode()), pi(sel), ri(n), pz(t1), ri(n),
                        pz(vr1), ri(n), pz(vr1), ri(n), ri(n), C.byref(m), pz(np.zeros(2 * n, complex)),
                        pz(np.zeros(n)), C.byref(info), C.c_size_t(1), C.c_size_t(1))
        mm = pkg.lib().arpack_hip_kit_ztrevc(C.c_char(howmny.encode()), pi(sel.copy()), n, pz(t2), n,
                                             pz(vr2), n)
        assert mm == m.value == n
        np.testing.assert_allclose(vr2, vr1, rtol=0, atol=1e-10)


@pytest.mark.parametrize("n,seed", [(12, 5), (30, 6)])
def test_ztrsen_matches_lapack(pkg, n, seed):
    B = _blas()
    t, z, w = _schur(pkg, _hess(n, seed))
    sel = np.zeros(n, np.int32)
    sel[np.random.default_rng(seed).permutation(n)[:n // 3]] = 1
    t1, q1, w1 = t.copy(order="F"), z.copy(order="F"), np.zeros(n, complex)
    m1, info1 = C.c_int(), C.c_int()
    B.scipy_ztrsen_(C.c_char_p(b"N"), C.c_char_p(b"V"), pi(sel), ri(n), pz(t1), ri(n), pz(q1), ri(n),
                    pz(w1), C.byref(m1), C.byref(C.c_double()), C.byref(C.c_double()),
                    pz(np.zeros(n, complex)), ri(n), C.byref(info1), C.c_size_t(1), C.c_size_t(1))
    t2, q2, w2 = t.copy(order="F"), z.copy(order="F"), np.zeros(n, complex)
    m2 = C.c_int()
    assert pkg.lib().arpack_hip_kit_ztrsen(pi(sel), n, pz(t2), n, pz(q2), n, pz(w2), C.byref(m2)) == 0
    assert m1.value == m2.value and info1.value == 0
    np.testing.assert_allclose(w2, w1, rtol=0, atol=1e-12 * np.abs(w1).max())
    np.testing.assert_allclose(q2, q1, rtol=0, atol=1e-11)


@needs_ref
@pytest.mark.parametrize("which", ["LM", "SM", "LR", "SR", "LI", "SI"])
def test_zsortc_zngets_match_reference(pkg, which):
    rng = np.random.default_rng(9)
    n = 29
    x = np.round(rng.standard_normal(n), 1) + 1j * np.round(rng.standard_normal(n), 1)
    y = np.arange(n).astype(complex)
    a = [x.copy(), y.copy()]
    ref.lib().zsortc_(C.c_char_p(which.encode()), ri(1), ri(n), pz(a[0]), pz(a[1]), C.c_size_t(2))
    b = [x.copy(), y.copy()]
    pkg.lib().arpack_hip_kit_zsortc(which.encode(), 1, n, pz(b[0]), pz(b[1]))
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    for ishift in (0, 1):
        a = [x.copy(), y.copy()]
        ref.lib().zngets_(ri(ishift), C.c_char_p(which.encode()), ri(10), ri(n - 10), pz(a[0]), pz(a[1]),
                          C.c_size_t(2))
        b = [x.copy(), y.copy()]
        pkg.lib().arpack_hip_kit_zngets(ishift, which.encode(), 10, n - 10, pz(b[0]), pz(b[1]))
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


@needs_ref
@pytest.mark.parametrize("n,seed", [(10, 0), (30, 1)])
def test_zneigh_matches_reference(pkg, n, seed):
    h = _hess(n, seed + 20)
    r1, b1, q1 = np.zeros(n, complex), np.zeros(n, complex), np.zeros((n, n), complex, order="F")
    ierr = C.c_int()
    ref.lib().zneigh_(C.byref(C.c_double(0.37)), ri(n), pz(h.copy(order="F")), ri(n), pz(r1), pz(b1),
                      pz(q1), ri(n), pz(np.zeros(n * n + 3 * n, complex)), pz(np.zeros(n)), C.byref(ierr))
    r2, b2, q2 = np.zeros(n, complex), np.zeros(n, complex), np.zeros((n, n), complex, order="F")
    assert pkg.lib().arpack_hip_kit_zneigh(C.c_double(0.37), n, pz(h), n, pz(r2), pz(b2), pz(q2), n) == 0
    assert ierr.value == 0
    np.testing.assert_allclose(r2, r1, rtol=0, atol=1e-12 * np.abs(r1).max())
    np.testing.assert_allclose(np.abs(b2), np.abs(b1), rtol=0, atol=1e-10 * np.abs(b1).max())


@needs_ref
@pytest.mark.parametrize("kev,seed", [(10, 0), (4, 1)])
def test_znapps_host_matches_reference(pkg, kev, seed):
    kp = 30 if kev == 10 else 12
    n = 50
    h = _hess(kp, seed + 40)
    h[np.arange(1, kp), np.arange(kp - 1)] = np.abs(h[np.arange(1, kp), np.arange(kp - 1)])
    rng = np.random.default_rng(seed)
    shift = rng.standard_normal(kp - kev) + 1j * rng.standard_normal(kp - kev) + 3.0
    h1, h2 = h.copy(order="F"), h.copy(order="F")
    q1, q2 = (np.zeros((kp, kp), complex, order="F") for _ in range(2))
    v = np.asfortranarray(rng.standard_normal((n, kp)) + 0j)
    ref.lib().znapps_(ri(n), ri(kev), ri(kp - kev), pz(shift), pz(v), ri(n), pz(h1), ri(kp),
                      pz(np.ones(n, complex)), pz(q1), ri(kp), pz(np.zeros(kp, complex)),
                      pz(np.zeros(2 * n, complex)))
    pkg.lib().arpack_hip_kit_znapps_host(kev, kp - kev, pz(shift), pz(h2), kp, pz(q2), kp, C.c_int64(n))
    np.testing.assert_allclose(h2, h1, rtol=0, atol=1e-10 * np.abs(h1).max())
    np.testing.assert_allclose(q2, q1, rtol=0, atol=1e-10)
