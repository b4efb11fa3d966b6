"""CPU: the engine's host small-dense kit (restated LAPACK/ARPACK ncv-sized
routines) against the REAL reference's internal routines (oracle/_ref) and the
image's LAPACK, on the same inputs."""
import ctypes as C

import numpy as np
import pytest

from oracle import matrices as M
from oracle import ref

needs_ref = pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built")
pd = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
pi = lambda a: a.ctypes.data_as(C.POINTER(C.c_int))  # noqa: E731


def _blas():
    import glob, os, scipy
    p = glob.glob(os.path.join(os.path.dirname(scipy.__file__), "..", "scipy.libs",
                               "libscipy_openblas*.so"))[0]
    return C.CDLL(p)


def test_dlartg_matches_lapack(pkg):
    L = pkg.lib()
    B = _blas()
    rng = np.random.default_rng(0)
    cases = [(0.0, 0.0), (0.0, 2.0), (0.0, -3.0), (3.0, 0.0), (-1.0, 1.0), (1e-300, 1e-300),
             (1e300, 1e290), (-2.5, 7.25)] + [tuple(x) for x in rng.standard_normal((200, 2))]
    for f, g in cases:
        c, s, r = C.c_double(), C.c_double(), C.c_double()
        L.arpack_hip_kit_dlartg(f, g, C.byref(c), C.byref(s), C.byref(r))
        c2, s2, r2 = C.c_double(), C.c_double(), C.c_double()
        B.scipy_dlartg_(C.byref(C.c_double(f)), C.byref(C.c_double(g)), C.byref(c2), C.byref(s2),
                        C.byref(r2))
        assert (c.value, s.value, r.value) == (c2.value, s2.value, r2.value), (f, g)


def test_dlarnv_host_kit_matches_lapack(pkg, golden):
    g = golden("g7_dlarnv")
    iseed = np.array([1, 3, 5, 7], np.int32)
    x = np.zeros(1000)
    pkg.lib().arpack_hip_kit_dlarnv(pi(iseed), 1000, x.ctypes.data)
    assert np.array_equal(x, g["x"]) and np.array_equal(iseed, g["iseed_out"])
    y, s = M.dlarnv_uniform(1000)
    assert np.array_equal(y, g["x"]) and tuple(s) == tuple(g["iseed_out"])


def _digits(s48):
    return np.array([(s48 >> 36) & 4095, (s48 >> 24) & 4095, (s48 >> 12) & 4095, s48 & 4095],
                    np.int32)


@pytest.mark.parametrize("case", ["plain", "redraw_chunk1", "redraw_chunk3"])
def test_slarnv_host_kit_matches_lapack(pkg, case):
    """slarnv(idist=2) in float: LAPACK slaruv's REAL conversion, its 64-draw
    batches and its redraw rule when a draw rounds to 1.0 (every seed digit + 2),
    bit for bit against the image's LAPACK (scipy_slarnv_)."""
    a, m = 33952834046453, 1 << 48
    if case == "plain":
        seeds, n = [np.array([1, 3, 5, 7], np.int32), np.array([4095, 17, 2, 9], np.int32)], 1000
    else:
        # seed such that draw k (1-based, within the first batch or the third)
        # is 2^48 - 1, which REAL arithmetic rounds to exactly 1.0
        k = 5 if case == "redraw_chunk1" else 2 * 64 + 7
        s = ((m - 1) * pow(pow(a, k, m), -1, m)) % m
        seeds, n = [_digits(s)], 300
    B = _blas()
    for iseed in seeds:
        for nn in (n, 63, 64, 65):
            x1, s1 = np.zeros(nn, np.float32), iseed.copy()
            B.scipy_slarnv_(C.byref(C.c_int(2)), pi(s1), C.byref(C.c_int(nn)),
                            x1.ctypes.data_as(C.c_void_p))
            x2, s2 = np.zeros(nn, np.float32), iseed.copy()
            pkg.lib().arpack_hip_kit_slarnv(pi(s2), nn, x2.ctypes.data)
            assert np.array_equal(x1, x2), (case, nn, np.flatnonzero(x1 != x2)[:5])
            assert np.array_equal(s1, s2), (case, nn, s1, s2)
    if case != "plain":  # the redraw really happened: the closed form differs from there on
        y, _ = M.dlarnv_uniform(n, tuple(int(t) for t in seeds[0]))
        assert not np.array_equal(y.astype(np.float32), x1)


@needs_ref
@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (5, 2), (20, 3), (30, 4), (64, 5)])
def test_dstqrb_matches_reference(pkg, n, seed):
    rng = np.random.default_rng(seed)
    d = rng.standard_normal(n)
    e = np.abs(rng.standard_normal(max(n - 1, 1)))
    if n > 4:
        e[n // 3] = 0.0  # a split
    L = ref.lib()
    d1, e1, z1, w1 = d.copy(), e.copy(), np.zeros(n), np.zeros(max(2 * n - 2, 1))
    info1 = np.zeros(1, np.int32)
    L.dstqrb_(C.byref(C.c_int(n)), pd(d1), pd(e1), pd(z1), pd(w1), pi(info1))
    d2, e2, z2, w2 = d.copy(), e.copy(), np.zeros(n), np.zeros(max(2 * n - 2, 1))
    info2 = pkg.lib().arpack_hip_kit_dstqrb(n, d2.ctypes.data, e2.ctypes.data, z2.ctypes.data,
                                            w2.ctypes.data)
    assert info1[0] == info2 == 0
    np.testing.assert_array_equal(d1, d2)
    np.testing.assert_array_equal(z1, z2)


@pytest.mark.parametrize("n", [1, 3, 10, 30])
def test_dsteqr_matches_lapack(pkg, n):
    rng = np.random.default_rng(n)
    d = rng.standard_normal(n)
    e = rng.standard_normal(max(n - 1, 1))
    B = _blas()
    d1, e1 = d.copy(), e.copy()
    z1 = np.zeros((n, n), order="F")
    w1 = np.zeros(max(2 * n - 2, 1))
    info = np.zeros(1, np.int32)
    B.scipy_dsteqr_(C.c_char_p(b"I"), C.byref(C.c_int(n)), pd(d1), pd(e1), pd(z1),
                    C.byref(C.c_int(n)), pd(w1), pi(info), C.c_size_t(1))
    d2, e2 = d.copy(), e.copy()
    z2 = np.zeros((n, n), order="F")
    w2 = np.zeros(max(2 * n - 2, 1))
    assert pkg.lib().arpack_hip_kit_dsteqr(n, d2.ctypes.data, e2.ctypes.data, z2.ctypes.data, n,
                                           w2.ctypes.data) == 0
    np.testing.assert_allclose(d2, d1, rtol=0, atol=1e-14 * max(1, np.abs(d1).max()))
    # eigenvectors up to sign
    for k in range(n):
        s = np.sign(z1[:, k] @ z2[:, k]) or 1.0
        np.testing.assert_allclose(s * z2[:, k], z1[:, k], atol=1e-12)


@needs_ref
@pytest.mark.parametrize("which", ["LA", "SA", "LM", "SM"])
def test_dsortr_tie_order_matches_reference(pkg, which):
    rng = np.random.default_rng(7)
    x = np.round(rng.standard_normal(37), 1)  # many ties, both signs
    y = np.arange(37, dtype=np.float64)
    x1, y1 = x.copy(), y.copy()
    ref.lib().dsortr_(C.c_char_p(which.encode()), C.byref(C.c_int(1)), C.byref(C.c_int(37)),
                      pd(x1), pd(y1), C.c_size_t(2))
    x2, y2 = x.copy(), y.copy()
    pkg.lib().arpack_hip_kit_dsortr(which.encode(), 1, 37, x2.ctypes.data, y2.ctypes.data)
    np.testing.assert_array_equal(x1, x2)
    np.testing.assert_array_equal(y1, y2)


@needs_ref
@pytest.mark.parametrize("kev,np_,seed", [(10, 20, 0), (4, 16, 1), (1, 5, 2), (15, 15, 3)])
def test_dsapps_rotations_match_reference(pkg, kev, np_, seed):
    """Host bulge chase + Q accumulation of dsapps vs the reference dsapps_ (n small)."""
    rng = np.random.default_rng(seed)
    kp = kev + np_
    n = 50
    h = np.zeros((kp, 2), order="F")
    h[1:, 0] = np.abs(rng.standard_normal(kp - 1)) + 0.1
    h[:, 1] = rng.standard_normal(kp)
    if kp > 6:
        h[kp // 2, 0] = 1e-300  # force a deflation
    shifts = rng.standard_normal(np_)
    v = np.asfortranarray(rng.standard_normal((n, kp)))
    resid = rng.standard_normal(n)
    q1 = np.zeros((kp, kp), order="F")
    h1 = h.copy(order="F")
    workd = np.zeros(2 * n)
    ref.lib().dsapps_(C.byref(C.c_int(n)), C.byref(C.c_int(kev)), C.byref(C.c_int(np_)),
                      pd(shifts), pd(v), C.byref(C.c_int(n)), pd(h1), C.byref(C.c_int(kp)),
                      pd(resid), pd(q1), C.byref(C.c_int(kp)), pd(workd))
    h2 = h.copy(order="F")
    q2 = np.zeros((kp, kp), order="F")
    pkg.lib().arpack_hip_kit_dsapps_host(kev, np_, shifts.ctypes.data, h2.ctypes.data, kp,
                                         q2.ctypes.data, kp)
    np.testing.assert_array_equal(h1, h2)
    np.testing.assert_array_equal(q1, q2)
