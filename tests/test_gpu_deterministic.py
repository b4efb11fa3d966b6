"""GPU: deterministic mode (arpack_hip_set_deterministic; VERDICT r03 weak #6,
r04 weak #5).

The default upper-triangle symmetric SpMV and the complex row-tile SpMV
accumulate in LDS with atomics in wave-schedule order, so a solve through them
reproduces its Ritz values to ~1e-15 but not bit for bit.  Deterministic mode
keeps only fixed-order forms: the symmetric declaration takes the fixed-point
form of the upper-triangle kernel (k_csr_ssell_det: the transposed terms summed
as exact 64-bit integers, the row sums in lane order), the complex operator the
column-split kernel.  Repeated products and solves must then agree BITWISE,
under uneven load too; the fixed-point product stays within its stated bound
of SciPy's (64 eps (|A||x|)_i for the row part plus 2^-50 amax max|x| a
transposed term); an operator outside the form keeps full storage (rc = 1).
"""
import ctypes as C

import numpy as np
import pytest

from oracle import matrices as M

pytestmark = pytest.mark.gpu


@pytest.fixture
def det(pkg):
    pkg.set_deterministic(True)
    yield
    pkg.set_deterministic(False)


def test_symmetric_declaration_takes_fixed_point_form(pkg, det):
    A = pkg.CSR.banded_sym(200_000, 1234, 4096, 25)
    A.set_symmetric(True)
    assert A.last_rc == 0 and A.symmetric
    n = A.n
    v0 = M.dlarnv_uniform(n)[0]
    runs = []
    for _ in range(3):
        s = pkg.SymRci(n, 10, 30, "LA", 1e-8, mxiter=300, device=True, v0=v0)
        assert s.aupd_csr(A) == 99 and int(s.info[0]) == 0
        d, z, nconv = s.eupd(rvec=True)
        runs.append((int(s.iparam[2]), int(s.iparam[8]), d[:nconv].copy(),
                     z.numpy()[: nconv * n].copy()))
    for r in runs[1:]:
        assert r[:2] == runs[0][:2]
        np.testing.assert_array_equal(r[2], runs[0][2])  # bitwise
        np.testing.assert_array_equal(r[3], runs[0][3])
    # the same solve through the full-storage SpMV (bitwise csr_matvec): same
    # cycles and OP*x, Ritz values to rounding
    A.set_symmetric(False)
    s = pkg.SymRci(n, 10, 30, "LA", 1e-8, mxiter=300, device=True, v0=v0)
    assert s.aupd_csr(A) == 99 and int(s.info[0]) == 0
    d, _, nconv = s.eupd(rvec=False)
    assert (int(s.iparam[2]), int(s.iparam[8])) == runs[0][:2]
    np.testing.assert_allclose(np.sort(d[:nconv]), np.sort(runs[0][2]), rtol=1e-12)


N, BAND, PER_ROW = 2_000_000, 4096, 25


def _hook(pkg):
    f = pkg.lib().arpack_hip_test_symspmv_handoff
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int64,
                  C.c_void_p, C.c_int64, C.c_void_p]
    return f


def _bound(S, x):
    """64 eps (|A||x|)_i for the row sums, plus (L + 1) 2^-50 amax max|x| for
    the transposed terms (L: the most entries left of the diagonal in a row;
    each term rounded to 2^(E-B) <= 2^-50 amax max|x|, B = 51)."""
    import scipy.sparse as sp
    U = sp.triu(S, 1)
    L = int(np.diff(sp.tril(S, -1).tocsr().indptr).max())
    amax = float(abs(U).max())
    return (64 * np.finfo(float).eps * (abs(S) @ np.abs(x))
            + (L + 1) * 2.0 ** -50 * amax * np.abs(x).max())


@pytest.mark.parametrize("fuse", [0, 1])
def test_fixed_point_spmv_bitwise_under_uneven_load(pkg, det, fuse):
    """The product itself, repeated while a read / write stream occupies the
    CUs from another stream (uneven arrival; the fused form's chain-head
    hand-off included): every run bitwise equal to the first, and within the
    bound of SciPy's product -- with x spread over eight decades, so the
    fixed-point scale (the window's largest |x|) is far above most terms."""
    import scipy.sparse as sp
    A = pkg.CSR.banded_sym(N, 99, BAND, PER_ROW)
    rp, col, val = A.download()
    A.set_symmetric(True)
    assert A.last_rc == 0 and A.symmetric
    S = sp.csr_matrix((val, col, rp), shape=(N, N))
    rng = np.random.default_rng(8)
    x = rng.standard_normal(N) * 10.0 ** rng.uniform(-8, 0, N)
    bound = _bound(S, x)
    xd = pkg.DeviceBuffer.from_numpy(x)
    xbig = pkg.DeviceBuffer.from_numpy(x * 1e12)
    load = pkg.DeviceBuffer(256 * 1024 * 1024 // 8)
    heads = np.zeros(2 * 4096, np.int64)
    f = _hook(pkg)
    yd = pkg.DeviceBuffer(N)
    y0 = None
    for rep in range(8):
        if rep % 2:  # a product of another scale first: its running maximum is
            # left in LDS, and must not leak into the next launch's scale
            f(A.h, xbig.ptr, yd.ptr, fuse, None, 0, heads.ctypes.data, 4096, None)
        pkg.lib().arpack_hip_memset(yd.ptr, 0xFF, 8 * N)  # NaN: an unwritten row cannot pass
        rc = f(A.h, xd.ptr, yd.ptr, fuse, load.ptr if rep else None, load.n if rep else 0,
               heads.ctypes.data, 4096, None)
        assert rc > 0, rc
        y = yd.numpy()
        if y0 is None:
            y0 = y.copy()
            err = np.abs(y - S @ x)
            assert np.all(err <= bound), (int((err > bound).sum()), float((err / bound).max()))
        else:
            np.testing.assert_array_equal(y.view(np.int64), y0.view(np.int64))


def test_fixed_point_spmv_wide_superblocks(pkg, det):
    """A narrow band (16) gives superblocks of ~7,800 rows (123 slices: more
    than 6 a wave, the kernel's 10-slice instance): bitwise repeatable and
    within the bound, both with and without the fused combine."""
    import scipy.sparse as sp
    n = 2_000_000
    A = pkg.CSR.banded_sym(n, 11, 16, 6)
    rp, col, val = A.download()
    A.set_symmetric(True)
    assert A.last_rc == 0 and A.symmetric
    S = sp.csr_matrix((val, col, rp), shape=(n, n))
    x = np.random.default_rng(2).standard_normal(n)
    bound = _bound(S, x)
    xd, yd = pkg.DeviceBuffer.from_numpy(x), pkg.DeviceBuffer(n)
    heads = np.zeros(2 * 4096, np.int64)
    f = _hook(pkg)
    ys = []
    for fuse in (0, 1, 0, 1):
        assert f(A.h, xd.ptr, yd.ptr, fuse, None, 0, heads.ctypes.data, 4096, None) > 0
        ys.append(yd.numpy().copy())
    assert np.all(np.abs(ys[0] - S @ x) <= bound)
    for y in ys[1:]:
        np.testing.assert_array_equal(y.view(np.int64), ys[0].view(np.int64))


def test_fixed_point_spmv_propagates_nan(pkg, det):
    """A NaN in x reaches y: every row SciPy's product makes NaN is NaN here
    too (the scale of a window holding a NaN is NaN)."""
    import scipy.sparse as sp
    n = 300_000
    A = pkg.CSR.banded_sym(n, 5, BAND, PER_ROW)
    rp, col, val = A.download()
    A.set_symmetric(True)
    assert A.symmetric
    S = sp.csr_matrix((val, col, rp), shape=(n, n))
    x = np.linspace(-1.0, 1.0, n)
    x[123_457] = np.nan
    y = np.empty(n)
    xd, yd = pkg.DeviceBuffer.from_numpy(x), pkg.DeviceBuffer(n)
    A.matvec_device(xd, yd)
    y = yd.numpy()
    with np.errstate(invalid="ignore"):
        ref = S @ x
    assert np.isnan(ref).sum() > 1
    assert np.all(np.isnan(y[np.isnan(ref)]))


def test_full_window_keeps_full_storage(pkg, det):
    """A superblock window that fills all 10,240 LDS columns leaves no word for
    the running maximum: the declaration keeps the full-storage kernel and
    reports it (rc = 1), as for any operator outside the fixed-point form."""
    n = 20_000
    i = np.arange(n)
    rows = np.concatenate([i, i[1:], i[:-1], [0, 10_239]])
    cols = np.concatenate([i, i[:-1], i[1:], [10_239, 0]])
    vals = np.concatenate([np.full(n, 2.0), np.full(2 * (n - 1), -1.0), [0.5, 0.5]])
    import scipy.sparse as sp
    S = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    S.sort_indices()
    A = pkg.CSR.from_arrays(S.indptr, S.indices, S.data)
    A.set_symmetric(True)
    assert A.last_rc == 1 and not A.symmetric
    pkg.set_deterministic(False)
    A.set_symmetric(True)  # the default kernel takes the same plan
    assert A.last_rc == 0 and A.symmetric
    pkg.set_deterministic(True)


def test_declared_first_then_deterministic_runs_full_storage(pkg):
    """an operator declared symmetric while deterministic
    mode is off, whose fixed-point form is NOT available (the full-window
    operator above: ss_det = 0), keeps the LDS-atomic kernel -- until the mode
    is switched on: its products then run the full-storage fixed-order kernel
    (the full CSR stays resident), so they repeat bitwise and equal the
    full-storage product bit for bit; switching the mode off restores the
    symmetric kernel."""
    import scipy.sparse as sp
    n = 20_000
    i = np.arange(n)
    rows = np.concatenate([i, i[1:], i[:-1], [0, 10_239]])
    cols = np.concatenate([i, i[:-1], i[1:], [10_239, 0]])
    vals = np.concatenate([np.full(n, 2.0), np.full(2 * (n - 1), -1.0), [0.5, 0.5]])
    S = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    S.sort_indices()
    x = np.random.default_rng(4).standard_normal(n) * 10.0 ** np.random.default_rng(5).uniform(-6, 0, n)
    xd, yd = pkg.DeviceBuffer.from_numpy(x), pkg.DeviceBuffer(n)
    F = pkg.CSR.from_arrays(S.indptr, S.indices, S.data)  # full storage throughout
    F.matvec_device(xd, yd)
    y_full = yd.numpy().copy()
    pkg.set_deterministic(False)
    A = pkg.CSR.from_arrays(S.indptr, S.indices, S.data)
    A.set_symmetric(True)
    assert A.last_rc == 0 and A.symmetric
    try:
        pkg.set_deterministic(True)
        ys = []
        for _ in range(4):
            pkg.lib().arpack_hip_memset(yd.ptr, 0xFF, 8 * n)
            A.matvec_device(xd, yd)
            ys.append(yd.numpy().copy())
        for y in ys:
            np.testing.assert_array_equal(y.view(np.int64), y_full.view(np.int64))
        # and a (capped) solve through it is bitwise repeatable
        v0 = M.dlarnv_uniform(n)[0]
        runs = []
        for _ in range(2):
            s = pkg.SymRci(n, 4, 20, "LA", 1e-10, mxiter=20, device=True, v0=v0)
            assert s.aupd_csr(A) == 99 and int(s.info[0]) in (0, 1)
            o5 = int(s.ipntr[5]) - 1
            runs.append((int(s.iparam[2]), int(s.iparam[8]), s.workl[o5:o5 + 20].copy()))
        assert runs[0][:2] == runs[1][:2]
        np.testing.assert_array_equal(runs[0][2], runs[1][2])
    finally:
        pkg.set_deterministic(False)
    A.matvec_device(xd, yd)  # the symmetric kernel again: SciPy's product to rounding
    np.testing.assert_allclose(yd.numpy(), S @ x, rtol=0, atol=1e-12 * np.abs(x).max() * 4)


def test_deterministic_off_restores_symmetric(pkg):
    pkg.set_deterministic(False)
    A = pkg.CSR.banded_sym(200_000, 1234, 4096, 25)
    A.set_symmetric(True)
    assert A.last_rc == 0 and A.symmetric


def test_complex_operator_bitwise_repeatable(pkg, det):
    n = 100_000
    Z = pkg.ZCSR.random(n, 100, 5, 100.0)
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)
    x = (np.arange(n) % 7 - 3.0) + 1j * (np.arange(n) % 5 - 2.0)
    y0 = Z.matvec(x)
    for _ in range(3):
        np.testing.assert_array_equal(Z.matvec(x), y0)
    runs = []
    for _ in range(2):
        s = pkg.ZRci(n, 6, 20, "LM", 1e-8, mxiter=6, v0=v0)  # capped: Ritz values in workl
        s.aupd_zcsr(Z)
        runs.append((int(s.iparam[2]), np.array(s.ritz)))
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])


def test_complex_tiles_fixed_point_bitwise(pkg, det):
    """Config 5's operator family at a size that takes the XCD split with
    column-sorted tiles (n >= 2^18, >= 32 entries a row): deterministic mode
    runs the tiles' fixed-point form (k_ztile_det: row sums as exact 64-bit
    integers) -- bitwise equal products with products of another scale in
    between, within 64 eps (|A||x|) + (L + 1) 2^-49 amax max|x| of SciPy's per
    component -- and the default mode's LDS-atomic tiles agree to rounding."""
    import scipy.sparse as sp
    n = 300_000
    Z = pkg.ZCSR.random(n, 40, 7, 40.0)
    rp, col, val = Z.download()
    S = sp.csr_matrix((val, col, rp), shape=(n, n))
    rng = np.random.default_rng(4)
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 10.0 ** rng.uniform(-6, 0, n)
    y0 = Z.matvec(x)
    for k in range(4):
        Z.matvec(x * 1e9 if k % 2 else x[::-1].copy())
        np.testing.assert_array_equal(Z.matvec(x).view(np.int64), y0.view(np.int64))
    amax = max(np.abs(val.real).max(), np.abs(val.imag).max())
    L = int(np.diff(rp).max())
    xm = max(np.abs(x.real).max(), np.abs(x.imag).max())
    ref = S @ x
    bound = 64 * np.finfo(float).eps * (abs(S) @ np.abs(x)) + (L + 1) * 2.0 ** -49 * amax * xm
    assert np.all(np.abs(y0.real - ref.real) <= bound)
    assert np.all(np.abs(y0.imag - ref.imag) <= bound)
    pkg.set_deterministic(False)
    y1 = Z.matvec(x)
    pkg.set_deterministic(True)
    assert np.all(np.abs(y1 - y0) <= 2 * bound)
