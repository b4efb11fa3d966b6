"""CPU: the arithmetic of deterministic mode's fixed-point sums
(spmv_sym.hip k_csr_ssell_det, zsplit.hip k_ztile_det), restated in numpy.

Each term p becomes q = rint(p 2^(B-E)) through ONE fma onto M = 1.5 * 2^52:
the low mantissa bits of fma(p, 2^(B-E), M) are q (two's complement after
subtracting M's bit pattern) whenever |p 2^(B-E)| < 2^51.  Here p * 2^(B-E) is
exact (a power-of-two scale), so numpy's p * inv + M has the same single
rounding as the kernel's fma.  Checked: the conversion equals np.rint (ties
to even, negative values), integer sums are the same in every order, and the
reconstructed sum stays within L * 2^(E-B-1) of the exact one (the bound the
GPU tests use, with a 2x margin)."""
import numpy as np

M = 1.5 * 2.0 ** 52
MB = np.array([M]).view(np.int64)[0]


def to_fixed(p, inv):
    d = p * inv + M  # one rounding: p * inv is exact
    return d.view(np.int64) - MB


def test_magic_conversion_is_rint():
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.uniform(-2.0 ** 50, 2.0 ** 50, 100_000),
                        np.arange(-8, 8) + 0.5,  # ties: to even
                        [0.0, -0.0, 2.0 ** 51 - 1, -(2.0 ** 51 - 1)]])
    np.testing.assert_array_equal(to_fixed(v, 1.0), np.rint(v).astype(np.int64))


def test_sums_order_free_and_bounded():
    rng = np.random.default_rng(1)
    B, L = 51, 50
    amax, xmax = 0.37, 3.2e-4
    ea, ex = np.frexp(amax)[1], np.frexp(xmax)[1]
    E = int(ea + ex)
    inv, sc = 2.0 ** (B - E), 2.0 ** (E - B)
    for _ in range(200):
        a = rng.uniform(-amax, amax, L)
        x = rng.uniform(-xmax, xmax, L) * 10.0 ** rng.uniform(-12, 0, L)
        p = a * x
        assert np.all(np.abs(p * inv) < 2.0 ** B)
        q = to_fixed(p, inv)
        s1 = int(np.sum(q))
        s2 = int(np.sum(q[rng.permutation(L)]))
        assert s1 == s2  # integer addition: no order dependence
        exact = float(np.sum(p.astype(np.longdouble)))
        assert abs(s1 * sc - exact) <= L * 2.0 ** (E - B - 1) * 2


def test_scale_floor_keeps_terms_finite():
    """The kernels floor E at B - 1000 (inv <= 2^1000) and accept amax in
    [2^-900, 2^900]: xs = x_i * inv (the kernel's order: x scaled first, then
    the fma with a_ij) stays finite and every |a_ij xs| < 2^B whenever the
    products themselves are finite doubles (amax X < 2^1023)."""
    B = 51
    for amax in (2.0 ** -900, 1.0, 2.0 ** 900):
        for X in (2.0 ** -1000, 1e-300, 1.0, 1e120, 1e300):
            ea, ex = np.frexp(amax)[1], np.frexp(X)[1]
            if ea + ex > 1023:  # the products overflow in any arithmetic
                continue
            E = max(int(ea + ex), B - 1000)
            inv = 2.0 ** (B - E)
            xs = X * inv
            assert np.isfinite(xs) and abs(amax * xs) < 2.0 ** B
