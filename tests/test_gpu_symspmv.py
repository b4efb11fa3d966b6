"""GPU: symmetric-storage SpMV (arpack_hip_csr_set_symmetric, spmv_sym.hip).

The kernel streams only the upper triangle and gets the lower half from the
transposed terms, summed in one of two accumulators (one walk, k_csr_ssell):
the fixed-point form (default since round 6: exact 64-bit integer sums, y
bitwise reproducible run to run, each term rounded to 2^-51 of the window's
largest product) and the LDS fp64 atomics (schedule order, y reproducible to
~1 ulp; arpack_hip_csr_set_sym_accumulator(A, 1)).  Neither is bitwise SciPy's
(the full-storage kernel is, tests/test_gpu_parity.py::
test_spmv_bitwise_equals_scipy).  Bar here: |y - A@x| <= 64 eps (|A| |x|),
plus (L + 1) 2^-50 amax max|x| for the fixed-point form (L: the most
transposed terms a column receives), and whole solves on the reference's golden
fixtures with the SAME restart and OP*x counts and Ritz values within the
parity tolerance of test_gpu_parity.
"""
import numpy as np
import pytest

from oracle import matrices as M
from tests.test_gpu_parity import _check, _mat

pytestmark = pytest.mark.gpu

EPS = np.finfo(np.float64).eps


ACCS = ["fixed", "fp64"]


def _spmv_sym(pkg, rp, col, val, x, acc="fixed"):
    Ad = pkg.CSR.from_arrays(rp, col, val)
    Ad.set_symmetric(True)
    Ad.set_sym_accumulator(acc)
    xd = pkg.DeviceBuffer.from_numpy(x)
    yd = pkg.DeviceBuffer(len(rp) - 1)
    Ad.matvec_device(xd.at(0), yd.at(0))
    return yd.numpy(), Ad


def _fixed_term(rp, col, val, x):
    """(L + 1) 2^-50 amax max|x|: the fixed-point form's rounding of the
    transposed terms (L: strictly-upper entries of the column that receives
    the most; amax: the largest |a_ij| above the diagonal)."""
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    up = col > rows
    if not up.any():
        return 0.0
    L = int(np.bincount(col[up], minlength=len(rp) - 1).max())
    return (L + 1) * 2.0 ** -50 * float(np.abs(val[up]).max()) * float(np.abs(x).max())


def _close(rp, col, val, x, y, acc="fp64"):
    yref = M.to_scipy(rp, col, val) @ x
    scale = M.to_scipy(rp, col, np.abs(val)) @ np.abs(x)
    err = np.abs(y - yref)
    bound = 64 * EPS * scale + (_fixed_term(rp, col, val, x) if acc == "fixed" else 0.0)
    assert np.all(err <= bound), (err / np.maximum(bound, 1e-300)).max()


@pytest.mark.parametrize("spec", [("banded_sym", 20000, 1234, 512, 25),
                                  ("banded_sym", 40000, 99, 4096, 25),   # NS band: spills
                                  ("banded_sym", 3000, 5, 64, 3),
                                  ("laplace2d", 37, 3.0), ("laplace3d", 21, 1.0),
                                  ("anderson", 13, 3, 16.0, 1234), ("diag", 1000), ("diag", 1)])
@pytest.mark.parametrize("acc", ACCS)
def test_symmetric_spmv_matches_full(pkg, spec, acc):
    rp, col, val = _mat(spec)
    x = np.random.default_rng(3).standard_normal(len(rp) - 1)
    y, Ad = _spmv_sym(pkg, rp, col, val, x, acc)
    assert Ad.sym_form == ("sym_fixed" if acc == "fixed" else "sym_fp64")
    _close(rp, col, val, x, y, acc)


@pytest.mark.parametrize("acc", ACCS)
def test_symmetric_spmv_ns_shape_property(pkg, acc):
    """North-star operator family at 2e5 rows (band 4096, ~51 nnz/row), generated
    on device: symmetric storage agrees with the full-storage (bitwise-SciPy)
    kernel row by row."""
    n = 200_000
    A = pkg.CSR.banded_sym(n, 1234, 4096, 25)
    B = pkg.CSR.banded_sym(n, 1234, 4096, 25)
    B.set_symmetric(True)
    B.set_sym_accumulator(acc)
    x = np.random.default_rng(11).standard_normal(n)
    xd = pkg.DeviceBuffer.from_numpy(x)
    ya = pkg.DeviceBuffer(n)
    yb = pkg.DeviceBuffer(n)
    A.matvec_device(xd.at(0), ya.at(0))
    B.matvec_device(xd.at(0), yb.at(0))
    rp, col, val = A.download()
    scale = M.to_scipy(rp, col, np.abs(val)) @ np.abs(x)
    fx = _fixed_term(rp, col, val, x) if acc == "fixed" else 0.0
    assert np.all(np.abs(ya.numpy() - yb.numpy()) <= 64 * EPS * scale + fx)


@pytest.mark.parametrize("acc", ACCS)
@pytest.mark.parametrize("n,band", [(3_000_000, 512), (10_000_000, 4096)])
def test_symmetric_spmv_chained_superblocks(pkg, n, band, acc):
    """Sizes where the plan has whole multiples of the CU count of superblocks,
    so each workgroup walks a chain and carries spills in LDS (2 and 8 per
    chain here): agreement with the full-storage kernel row by row."""
    A = pkg.CSR.banded_sym(n, 1234, band, 25)
    xd = pkg.DeviceBuffer(n)
    x = np.random.default_rng(4).standard_normal(n)
    xd.write(x)
    ya = pkg.DeviceBuffer(n)
    yb = pkg.DeviceBuffer(n)
    A.matvec_device(xd.at(0), ya.at(0))
    A.set_symmetric(True)
    A.set_sym_accumulator(acc)
    A.matvec_device(xd.at(0), yb.at(0))
    a, b = ya.numpy(), yb.numpy()
    # |A| |x| bound from the device too: |x| through |A| is not available, so use
    # the row sums of |a_ij| <= 2 * 16 + 25 * 2 (generator bounds) times max |x|;
    # fixed point: <= 128 transposed terms a column, |a_ij| <= 1 off the diagonal
    bound = 64 * EPS * (np.abs(a) + 128.0 * np.abs(x).max())
    if acc == "fixed":
        bound = bound + 129 * 2.0 ** -50 * np.abs(x).max()
    assert np.all(np.abs(a - b) <= bound)
    del A


def test_symmetric_ignores_lower_triangle(pkg):
    """Entries below the diagonal are not read (upper fill mode): corrupting them
    leaves y unchanged."""
    rp, col, val = _mat(("banded_sym", 5000, 7, 300, 9))
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    bad = val.copy()
    bad[col < rows] = 1e300
    x = np.random.default_rng(1).standard_normal(len(rp) - 1)
    for acc in ACCS:
        y, _ = _spmv_sym(pkg, rp, col, bad, x, acc)
        _close(rp, col, val, x, y, acc)


def test_symmetric_refused_for_wide_band(pkg):
    """A band wider than the LDS window keeps the full-storage kernel."""
    import scipy.sparse as sp
    n = 20000
    A = (sp.eye(n, format="lil") * 4.0)
    A[0, 15000] = A[15000, 0] = -1.0   # reach 15000 > the 10240-column window
    A = A.tocsr()
    A.sort_indices()
    rp, col, val = A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data
    Ad = pkg.CSR.from_arrays(rp, col, val)
    with pytest.raises(RuntimeError):
        Ad.set_symmetric(True)
    x = np.random.default_rng(2).standard_normal(len(rp) - 1)
    xd = pkg.DeviceBuffer.from_numpy(x)
    yd = pkg.DeviceBuffer(len(rp) - 1)
    Ad.matvec_device(xd.at(0), yd.at(0))
    assert np.array_equal(yd.numpy(), M.to_scipy(rp, col, val) @ x)


@pytest.mark.parametrize("name", ["g2_icb_ds", "g3_anderson3d", "g4_banded", "g5_anderson2d_sa",
                                  "g6_anderson2d_be", "g10_anderson2d_sm"])
def test_solve_with_symmetric_storage(pkg, golden, name):
    """Whole dsaupd/dseupd solve on the GPU with the symmetric-storage OP: same
    restart cycles and OP*x count as the reference, Ritz values and residuals
    within the parity tolerance."""
    g = golden(name)
    rp, col, val = _mat(g["spec"])
    A = M.to_scipy(rp, col, val)
    Ad = pkg.CSR.from_arrays(rp, col, val)
    Ad.set_symmetric(True)
    d, z, res = pkg.eigsh(Ad, A.shape[0], int(g["nev"]), int(g["ncv"]), str(g["which"]),
                          float(g["tol"]), v0=g["v0"], mxiter=int(g["mxiter"]), device=True)
    _check(g, d, res, z, A)


@pytest.mark.parametrize("acc", ACCS)
def test_symmetric_storage_run_to_run(pkg, acc):
    """fp64 accumulator: the LDS adds land in schedule order, so repeated solves
    are not bitwise equal -- but on an NS-shaped operator (band 4096, spills
    across superblocks) three repeats of the same solve take the same restart
    cycles and OP*x, and their Ritz values agree to 1e-13 relative with each
    other and with the (bitwise reproducible) full-storage solve.  Fixed-point
    accumulator (the default): the three solves are bitwise equal.  The full-size
    measurement: tools/ttc_repeat.py."""
    n = 400_000
    A = pkg.CSR.banded_sym(n, 1234, 4096, 25, 0, n)
    A.set_sym_accumulator(acc)
    v0 = np.random.default_rng(3).uniform(-1, 1, n)
    res = {}
    for storage in ("full", "sym", "sym", "sym"):
        A.set_symmetric(storage == "sym")
        s = pkg.SymRci(n, 10, 30, "LA", 1e-8, mxiter=300, device=True, v0=v0)
        assert s.aupd_cycles(A, -1) == 99 and int(s.info[0]) == 0
        d, _, nconv = s.eupd(rvec=False)
        assert nconv == 10
        res.setdefault(storage, []).append((int(s.iparam[2]), int(s.iparam[8]), np.sort(d)))
    (c0, o0, d0), = res["full"]
    for c, o, d in res["sym"]:
        assert (c, o) == (c0, o0)
        assert np.max(np.abs(d - d0) / np.abs(d0)) <= 1e-13
    if acc == "fixed":
        for c, o, d in res["sym"][1:]:
            np.testing.assert_array_equal(d, res["sym"][0][2])


def test_graded_operator_keeps_fp64_accumulator(pkg):
    """the fixed-point form rounds every transposed term to 2^-51 of
    the window's largest product, so the DEFAULT accumulator takes it only when
    the upper off-diagonal magnitudes span at most 2^20.  A graded operator
    (D A D with D over twelve decades) keeps the fp64 form, whose small rows
    stay accurate relative to their own terms; deterministic mode still takes
    the fixed-point form, and the products meet their bounds."""
    import scipy.sparse as sp
    rp, col, val = _mat(("banded_sym", 20000, 7, 256, 9))
    n = len(rp) - 1
    d = 10.0 ** np.linspace(-12, 0, n)
    S = sp.diags(d) @ M.to_scipy(rp, col, val) @ sp.diags(d)
    S = sp.csr_matrix(S)
    S.sort_indices()
    grp, gcol, gval = S.indptr.astype(np.int64), S.indices.astype(np.int32), S.data
    x = np.random.default_rng(5).standard_normal(n)
    y, Ad = _spmv_sym(pkg, grp, gcol, gval, x)
    assert Ad.sym_form == "sym_fp64"
    _close(grp, gcol, gval, x, y, "fp64")
    pkg.set_deterministic(True)
    try:
        Ad.set_symmetric(True)
        assert Ad.sym_form == "sym_fixed"
        xd, yd = pkg.DeviceBuffer.from_numpy(x), pkg.DeviceBuffer(n)
        Ad.matvec_device(xd.at(0), yd.at(0))
        _close(grp, gcol, gval, x, yd.numpy(), "fixed")
    finally:
        pkg.set_deterministic(False)
