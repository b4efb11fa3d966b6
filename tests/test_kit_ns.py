"""CPU: the nonsymmetric host small-dense kit (dense_ns.cpp) against the REAL
reference's internal routines (oracle/_ref: SRC/dsortc.f, dngets.f, dneigh.f,
dnapps.f) and the image's LAPACK (dlahqr, dtrevc, dlanv2, dnrm2), on the same
inputs.  Scalar LAPACK restatements are compared bit for bit; routines whose
reference goes through BLAS-2 kernels (dgemv/dger inside dlarf, dtrevc 'B')
are compared to a few ulps, since the BLAS summation order is the library's."""
import ctypes as C
import glob
import os

import numpy as np
import pytest

from oracle import ref

needs_ref = pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built")
pd = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
pi = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))  # noqa: E731
ri = lambda v: C.byref(C.c_int(v))  # noqa: E731


def _blas():
    import scipy
    p = glob.glob(os.path.join(os.path.dirname(scipy.__file__), "..", "scipy.libs",
                               "libscipy_openblas*.so"))[0]
    return C.CDLL(p)


def _hess(n, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    h = np.triu(rng.standard_normal((n, n)), -1) * scale
    return np.asfortranarray(h)


def test_dnrm2_bitwise(pkg):
    B = _blas()
    B.scipy_dnrm2_.restype = C.c_double
    L = pkg.lib()
    L.arpack_hip_kit_dnrm2.restype = C.c_double
    rng = np.random.default_rng(0)
    for n in [1, 2, 3, 7, 30, 101]:
        for _ in range(50):
            x = rng.standard_normal(n) * np.exp(rng.uniform(-20, 20))
            a = B.scipy_dnrm2_(ri(n), pd(x), ri(1))
            b = L.arpack_hip_kit_dnrm2(n, pd(x))
            assert a == b


def test_dlanv2_bitwise(pkg):
    B = _blas()
    rng = np.random.default_rng(1)
    cases = [(1.0, 2.0, 0.0, 3.0), (1.0, 0.0, 2.0, 3.0), (2.0, 1.0, -1.0, 2.0),
             (1.0, 1e-17, -1e-17, 1.0), (0.0, 1.0, 1.0, 0.0)]
    cases += [tuple(rng.standard_normal(4)) for _ in range(300)]
    for cs in cases:
        r1 = [C.c_double(v) for v in cs] + [C.c_double() for _ in range(6)]
        B.scipy_dlanv2_(*[C.byref(v) for v in r1])
        r2 = [C.c_double(v) for v in cs] + [C.c_double() for _ in range(6)]
        pkg.lib().arpack_hip_kit_dlanv2(*[C.byref(v) for v in r2])
        assert [v.value for v in r1] == [v.value for v in r2], cs


@pytest.mark.parametrize("n,seed", [(6, 0), (20, 1), (30, 2), (40, 3), (41, 4)])
def test_dlahqr_matches_lapack(pkg, n, seed):
    B = _blas()
    h = _hess(n, seed)
    # full Schur form + Schur vectors, and the dneigh configuration (one Z row)
    for zrows in (n, 1):
        h1, h2 = h.copy(order="F"), h.copy(order="F")
        if zrows == n:
            z1 = np.asfortranarray(np.eye(n))
        else:
            z1 = np.zeros(n)
            z1[-1] = 1.0
        z2 = z1.copy(order="F")
        wr1, wi1, wr2, wi2 = (np.zeros(n) for _ in range(4))
        info = C.c_int()
        t = C.c_int(1)
        B.scipy_dlahqr_(C.byref(t), C.byref(t), ri(n), ri(1), ri(n), pd(h1), ri(n), pd(wr1),
                        pd(wi1), ri(1), ri(zrows), pd(z1), ri(zrows), C.byref(info))
        rc = pkg.lib().arpack_hip_kit_dlahqr(1, 1, n, 1, n, pd(h2), n, pd(wr2), pd(wi2), 1,
                                             zrows, pd(z2), zrows)
        assert rc == info.value == 0
        np.testing.assert_array_equal(wr1, wr2)
        np.testing.assert_array_equal(wi1, wi2)
        np.testing.assert_array_equal(h1, h2)
        np.testing.assert_array_equal(z1, z2)


@pytest.mark.parametrize("n,seed", [(8, 0), (20, 5), (40, 6)])
def test_dtrevc_matches_lapack(pkg, n, seed):
    B = _blas()
    h = _hess(n, seed)
    z = np.asfortranarray(np.eye(n))
    wr, wi = np.zeros(n), np.zeros(n)
    assert pkg.lib().arpack_hip_kit_dlahqr(1, 1, n, 1, n, pd(h), n, pd(wr), pd(wi), 1, n, pd(z),
                                           n) == 0
    assert np.any(wi != 0)
    for howmny in ("A", "B"):
        vr1 = z.copy(order="F")
        vr2 = z.copy(order="F")
        sel = np.zeros(n, np.int32)
        work = np.zeros(3 * n)
        m, info = C.c_int(), C.c_int()
        B.scipy_dtrevc_(C.c_char_p(b"R"), C.c_char_p(howmny.encode()), pi(sel), ri(n), pd(h),
                        ri(n), pd(vr1), ri(n), pd(vr1), ri(n), ri(n), C.byref(m), pd(work),
                        C.byref(info), C.c_size_t(1), C.c_size_t(1))
        mm = pkg.lib().arpack_hip_kit_dtrevc(C.c_char(howmny.encode()), pi(sel.copy()), n, pd(h),
                                             n, pd(vr2), n, pd(np.zeros(3 * n)))
        assert mm == m.value == n
        if howmny == "A":
            np.testing.assert_array_equal(vr1, vr2)
        else:  # back-transform goes through dgemv
            np.testing.assert_allclose(vr1, vr2, rtol=0, atol=1e-13)


@needs_ref
@pytest.mark.parametrize("which", ["LM", "SM", "LR", "SR", "LI", "SI"])
def test_dsortc_matches_reference(pkg, which):
    rng = np.random.default_rng(11)
    n = 31
    xr = np.round(rng.standard_normal(n), 1)
    xi = np.round(rng.standard_normal(n), 1) * (rng.uniform(size=n) < 0.5)
    y = np.arange(n, dtype=np.float64)
    a = [xr.copy(), xi.copy(), y.copy()]
    ref.lib().dsortc_(C.c_char_p(which.encode()), ri(1), ri(n), pd(a[0]), pd(a[1]), pd(a[2]),
                      C.c_size_t(2))
    b = [xr.copy(), xi.copy(), y.copy()]
    pkg.lib().arpack_hip_kit_dsortc(which.encode(), 1, n, pd(b[0]), pd(b[1]), pd(b[2]))
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)


def _ritz(pkg, n, seed):
    h = _hess(n, seed)
    rr, ri_, bd = np.zeros(n), np.zeros(n), np.zeros(n)
    q = np.zeros((n, n), order="F")
    wk = np.zeros(n * n + 3 * n)
    assert pkg.lib().arpack_hip_kit_dneigh(C.c_double(0.37), n, pd(h), n, pd(rr), pd(ri_),
                                           pd(bd), pd(q), n, pd(wk)) == 0
    return h, rr, ri_, bd, q


@needs_ref
@pytest.mark.parametrize("n,seed", [(10, 0), (30, 1), (40, 2)])
def test_dneigh_matches_reference(pkg, n, seed):
    h, rr2, ri2, bd2, q2 = _ritz(pkg, n, seed)
    rr1, ri1, bd1 = np.zeros(n), np.zeros(n), np.zeros(n)
    q1 = np.zeros((n, n), order="F")
    wk = np.zeros(n * n + 3 * n)
    ierr = C.c_int()
    ref.lib().dneigh_(C.byref(C.c_double(0.37)), ri(n), pd(h.copy(order="F")), ri(n), pd(rr1),
                      pd(ri1), pd(bd1), pd(q1), ri(n), pd(wk), C.byref(ierr))
    assert ierr.value == 0
    np.testing.assert_array_equal(rr1, rr2)
    np.testing.assert_array_equal(ri1, ri2)
    np.testing.assert_array_equal(q1, q2)
    # bounds = rnorm*|e_n' Q x| come from a dgemv 'T' (library summation order)
    np.testing.assert_allclose(bd1, bd2, rtol=0, atol=1e-13 * np.abs(bd1).max())


@needs_ref
@pytest.mark.parametrize("which", ["LM", "SM", "LR", "SR", "LI", "SI"])
@pytest.mark.parametrize("ishift", [0, 1])
def test_dngets_matches_reference(pkg, which, ishift):
    n = 40
    _, rr, ri_, bd, _ = _ritz(pkg, n, 3)
    for kev in (10, 13, 20):
        np_ = n - kev
        a = [rr.copy(), ri_.copy(), bd.copy()]
        k1, p1 = C.c_int(kev), C.c_int(np_)
        ref.lib().dngets_(ri(ishift), C.c_char_p(which.encode()), C.byref(k1), C.byref(p1),
                          pd(a[0]), pd(a[1]), pd(a[2]), pd(np.zeros(n)), pd(np.zeros(n)),
                          C.c_size_t(2))
        b = [rr.copy(), ri_.copy(), bd.copy()]
        k2, p2 = C.c_int(kev), C.c_int(np_)
        pkg.lib().arpack_hip_kit_dngets(ishift, which.encode(), C.byref(k2), C.byref(p2),
                                        pd(b[0]), pd(b[1]), pd(b[2]))
        assert (k1.value, p1.value) == (k2.value, p2.value)
        for u, v in zip(a, b):
            np.testing.assert_array_equal(u, v)


@needs_ref
@pytest.mark.parametrize("kev,seed", [(10, 0), (12, 1), (20, 2), (5, 3)])
def test_dnapps_host_matches_reference(pkg, kev, seed):
    """Shifts = the unwanted Ritz values of H moved off the spectrum by 0.37
    (complex pairs adjacent, as dngets leaves them); compares the transformed H,
    Q and the returned kev.  (With the exact Ritz values as shifts the chase is
    ill-conditioned: a 1e-16 relative perturbation of H changes its output at
    O(1) in either implementation, so entries are not comparable there.)"""
    kp = 40 if kev != 5 else 16
    n = 50  # dnapps caches smlnum from its first call's n: keep n fixed
    h, rr, ri_, bd, _ = _ritz(pkg, kp, seed)
    k, p = C.c_int(kev), C.c_int(kp - kev)
    pkg.lib().arpack_hip_kit_dngets(1, b"LM", C.byref(k), C.byref(p), pd(rr), pd(ri_), pd(bd))
    kev, np_ = k.value, p.value
    rr = rr + 0.37
    h1, h2 = h.copy(order="F"), h.copy(order="F")
    q1 = np.zeros((kp, kp), order="F")
    q2 = np.zeros((kp, kp), order="F")
    rng = np.random.default_rng(seed)
    v = np.asfortranarray(rng.standard_normal((n, kp)))
    resid = rng.standard_normal(n)
    kev1 = C.c_int(kev)
    ref.lib().dnapps_(ri(n), C.byref(kev1), ri(np_), pd(rr), pd(ri_), pd(v), ri(n), pd(h1),
                      ri(kp), pd(resid), pd(q1), ri(kp), pd(np.zeros(kp)), pd(np.zeros(2 * n)))
    kev2 = pkg.lib().arpack_hip_kit_dnapps_host(kev, np_, pd(rr), pd(ri_), pd(h2), kp, pd(q2), kp,
                                                pd(np.zeros(kp)), C.c_int64(n))
    assert kev1.value == kev2
    # complex-pair steps run dlarf (dgemv + dger): a few ulps of drift allowed
    np.testing.assert_allclose(h1, h2, rtol=0, atol=1e-10 * np.abs(h1).max())
    np.testing.assert_allclose(q1, q2, rtol=0, atol=1e-10)


@pytest.mark.parametrize("n,seed,pick", [(12, 0, "last"), (20, 1, "every3"), (30, 2, "last"),
                                         (40, 3, "rand"), (40, 4, "rand")])
def test_dtrsen_matches_lapack(pkg, n, seed, pick):
    """Schur reordering used by dneupd (SRC/dneupd.f:659): dtrsen('N','V') with
    dtrexc/dlaexc/dlasy2 underneath, bitwise against the image's LAPACK."""
    B = _blas()
    h = _hess(n, seed)
    z = np.asfortranarray(np.eye(n))
    wr, wi = np.zeros(n), np.zeros(n)
    assert pkg.lib().arpack_hip_kit_dlahqr(1, 1, n, 1, n, pd(h), n, pd(wr), pd(wi), 1, n, pd(z),
                                           n) == 0
    sel = np.zeros(n, np.int32)
    if pick == "last":
        sel[-n // 3:] = 1
    elif pick == "every3":
        sel[::3] = 1
    else:
        sel[np.random.default_rng(seed).permutation(n)[:n // 2]] = 1
    t1, q1 = h.copy(order="F"), z.copy(order="F")
    wr1, wi1 = np.zeros(n), np.zeros(n)
    m1, info1 = C.c_int(), C.c_int()
    s_, sep = C.c_double(), C.c_double()
    work = np.zeros(n)
    iwork = np.zeros(1, np.int32)
    B.scipy_dtrsen_(C.c_char_p(b"N"), C.c_char_p(b"V"), pi(sel), ri(n), pd(t1), ri(n), pd(q1),
                    ri(n), pd(wr1), pd(wi1), C.byref(m1), C.byref(s_), C.byref(sep), pd(work),
                    ri(n), pi(iwork), ri(1), C.byref(info1), C.c_size_t(1), C.c_size_t(1))
    t2, q2 = h.copy(order="F"), z.copy(order="F")
    wr2, wi2 = np.zeros(n), np.zeros(n)
    m2 = C.c_int()
    info2 = pkg.lib().arpack_hip_kit_dtrsen(pi(sel), n, pd(t2), n, pd(q2), n, pd(wr2), pd(wi2),
                                            C.byref(m2))
    assert (info1.value, m1.value) == (info2, m2.value)
    np.testing.assert_array_equal(wr1, wr2)
    np.testing.assert_array_equal(wi1, wi2)
    np.testing.assert_array_equal(t1, t2)
    np.testing.assert_array_equal(q1, q2)
