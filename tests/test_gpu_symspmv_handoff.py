"""GPU: the fused symmetric SpMV's cross-workgroup hand-off, word by word
(MI355X_MICROARCH.md: "test every hand-off under UNEVEN
load, consumer L1-warm, checking every word").

k_csr_ssell<..., FUSE=true> combines each chain's head rows inside the kernel:
the two workgroups of a pair store their partials to the slots with sc1
stores, drain them, add to the pair's counter, and the second arriver reads
both slots with sc1 loads.  Here the product runs repeatedly while a
read / write stream occupies the CUs from a second stream (the pairs arrive
unevenly), and EVERY row of y -- the chain-head rows combined through the
slots in particular -- is compared with the unfused form (separate combine
launch after a kernel boundary).  The two differ only by the order of the
LDS atomic adds of the transposed terms, so the bound is 64 eps (|A| |x|)
per row.  Sensitivity: the same check applied to y with one slot half read as
zero (what a stale slot would give) must fail on the head rows."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, BAND, PER_ROW = 2_000_000, 4096, 25
REPS = 24


def _hook(pkg):
    L = pkg.lib()
    f = L.arpack_hip_test_symspmv_handoff
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int64,
                  C.c_void_p, C.c_int64, C.c_void_p]
    return f


@pytest.mark.parametrize("acc", ["fp64", "fixed"])
def test_fused_handoff_every_word_under_uneven_load(pkg, acc):
    """Both accumulators share the walk and the hand-off: fp64 -- the fused and
    unfused forms differ by the LDS order (64 eps (|A||x|) a row); fixed point
    -- they must be bitwise equal."""
    A = pkg.CSR.banded_sym(N, 99, BAND, PER_ROW)
    rp, col, val = A.download()
    A.set_symmetric(True)
    A.set_sym_accumulator(acc)
    assert A.symmetric
    import scipy.sparse as sp
    S = sp.csr_matrix((val, col, rp), shape=(N, N))
    x = np.random.default_rng(8).standard_normal(N)
    bound = 64 * np.finfo(float).eps * (abs(S) @ np.abs(x))
    ref_bound = bound
    if acc == "fixed":  # against SciPy: + the fixed-point rounding; fused vs unfused: bitwise
        rows_ = np.repeat(np.arange(N), np.diff(rp))
        up = col > rows_
        L = int(np.bincount(col[up], minlength=N).max())
        ref_bound = bound + (L + 1) * 2.0 ** -50 * float(np.abs(val[up]).max()) * np.abs(x).max()
    xd = pkg.DeviceBuffer.from_numpy(x)
    load = pkg.DeviceBuffer(256 * 1024 * 1024 // 8)  # a 256 MB read / write stream
    f = _hook(pkg)
    heads = np.zeros(2 * 4096, np.int64)
    lo = np.zeros(N)
    yr = pkg.DeviceBuffer(N)
    nh = f(A.h, xd.ptr, yr.ptr, 0, None, 0, heads.ctypes.data, 4096, lo.ctypes.data)
    assert nh > 0, nh
    y_split = yr.numpy()
    rows = np.concatenate([np.arange(heads[2 * k], heads[2 * k] + heads[2 * k + 1])
                           for k in range(nh)])
    assert len(rows) > 0.1 * N  # the NS-like band: most chain-head rows are combined
    # the unfused form is SciPy's product to the LDS-order (fixed point: its) rounding
    assert np.all(np.abs(y_split - S @ x) <= ref_bound)
    yf = pkg.DeviceBuffer(N)
    for rep in range(REPS):
        pkg.lib().arpack_hip_memset(yf.ptr, 0xFF, 8 * N)  # NaN: an unwritten row cannot pass
        rc = f(A.h, xd.ptr, yf.ptr, 1, load.ptr, load.n, heads.ctypes.data, 4096, None)
        assert rc == nh, rc
        y = yf.numpy()
        if acc == "fixed":
            np.testing.assert_array_equal(y.view(np.int64), y_split.view(np.int64))
            continue
        bad = ~(np.abs(y - y_split) <= bound)
        assert not bad.any(), (rep, int(bad.sum()), np.flatnonzero(bad)[:8])
    # sensitivity: a stale (zero) slot half on the head rows is caught
    y_stale = y.copy()
    y_stale[rows] -= lo[rows]
    caught = ~(np.abs(y_stale[rows] - y_split[rows]) <= bound[rows])
    assert caught.mean() > 0.9, caught.mean()
