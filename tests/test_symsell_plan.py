"""CPU: the symmetric-storage SpMV plan (host half of arpack_hip_csr_set_symmetric,
spmv_sym.hip) -- no GPU needed.

* invariants of arpack_hip_kit_symsell_plan: superblocks tile the rows, every
  window holds its rows' upper columns within `win`, every spill lies inside the
  NEXT superblock (so each row has at most two partial sums);
* the plan's semantics: per-superblock windows of upper-triangle products,
  spill/prefix slots and the two-term combine reproduce A @ x (the arithmetic
  that k_csr_ssell + k_ssell_combine perform on the device);
* matrices that do not fit (band wider than the window) are refused.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import matrices as M


def _plan(pkg, cmax, win, spill_in=0, spill_out=0):
    L = pkg.lib()
    L.arpack_hip_kit_symsell_plan.argtypes = [C.c_int64, C.c_void_p, C.c_int, C.c_int64, C.c_int64,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    n = len(cmax)
    cm = np.ascontiguousarray(cmax, np.int32)
    nsb = np.zeros(1, np.int64)
    r0s = np.zeros(n + 1, np.int64)
    spans = np.zeros(n + 1, np.int32)
    pre = np.zeros(n + 1, np.int32)
    rc = L.arpack_hip_kit_symsell_plan(n, cm.ctypes.data, win, spill_in, spill_out, nsb.ctypes.data,
                                       r0s.ctypes.data, spans.ctypes.data, pre.ctypes.data)
    k = int(nsb[0])
    return rc, r0s[:k + 1], spans[:k], pre[:k]


def _upper_cmax(rp, col, coff=0):
    n = len(rp) - 1
    cmax = np.arange(n, dtype=np.int64)
    rows = np.repeat(np.arange(n), np.diff(rp))
    col = col.astype(np.int64) - coff
    up = col >= rows
    np.maximum.at(cmax, rows[up], col[up])
    return cmax


def _simulate(rp, col, val, x, r0s, spans, pre):
    """y from the plan exactly as the device computes it (up to summation order)."""
    n = len(rp) - 1
    y = np.zeros(n)
    nsb = len(spans)
    lo = {}
    hi = {}
    for b in range(nsb):
        r0, r1, span = r0s[b], r0s[b + 1], spans[b]
        yw = np.zeros(span)
        for i in range(r0, r1):
            for k in range(rp[i], rp[i + 1]):
                j = col[k]
                if j < i:
                    continue
                assert j - r0 < span          # the window holds every upper column
                yw[i - r0] += val[k] * x[j]
                if j != i:
                    yw[j - r0] += val[k] * x[i]
        R = r1 - r0
        hi[b] = yw[:pre[b]].copy()
        y[r0 + pre[b]:r1] = yw[pre[b]:R]
        if b + 1 < nsb:
            lo[b + 1] = yw[R:span].copy()
            assert len(lo[b + 1]) == pre[b + 1]
        else:
            assert span == R
    for b in range(1, nsb):
        y[r0s[b]:r0s[b] + pre[b]] = lo[b] + hi[b]
    return y


@pytest.mark.parametrize("spec,win", [(("banded", 3000, 1234, 200, 9), 512),
                                      (("banded", 3000, 7, 256, 5), 512),
                                      (("lap2d", 40), 128),
                                      (("anderson", 9), 256),
                                      (("diag", 500), 64)])
def test_symsell_plan_reproduces_spmv(pkg, spec, win):
    if spec[0] == "banded":
        rp, col, val = M.banded_sym(spec[1], spec[2], spec[3], spec[4])
    elif spec[0] == "lap2d":
        rp, col, val = M.laplace2d(spec[1], 1.0)
    elif spec[0] == "anderson":
        rp, col, val = M.anderson(spec[1], 3, 16.0, 1234)
    else:
        rp, col, val = M.diag(spec[1])
    n = len(rp) - 1
    rc, r0s, spans, pre = _plan(pkg, _upper_cmax(rp, col), win)
    assert rc == 0
    # invariants: tiling, windows, spill inside the next superblock
    assert r0s[0] == 0 and r0s[-1] == n and np.all(np.diff(r0s) > 0)
    R = np.diff(r0s)
    assert np.all(spans <= win) and np.all(spans >= R)
    assert pre[0] == 0
    assert np.all(pre[1:] == spans[:-1] - R[:-1]) and np.all(pre[1:] <= R[1:])
    assert spans[-1] == R[-1]
    x = np.random.default_rng(5).standard_normal(n)
    y = _simulate(rp, col, val, x, r0s, spans, pre)
    yref = M.to_scipy(rp, col, val) @ x
    scale = M.to_scipy(rp, col, np.abs(val)) @ np.abs(x)
    assert np.all(np.abs(y - yref) <= 1e-13 * scale + 1e-300)


def test_symsell_plan_refuses_wide_band(pkg):
    rp, col, val = M.banded_sym(2000, 1234, 600, 5)
    rc, *_ = _plan(pkg, _upper_cmax(rp, col), 512)   # a row reaches ~600 columns ahead
    assert rc == -1


def test_symsell_plan_edge_sizes(pkg):
    # one row, rows with no upper entries (cmax = i), one superblock
    for n in (1, 2, 63, 64, 65):
        rc, r0s, spans, pre = _plan(pkg, np.arange(n), 64)
        assert rc == 0 and r0s[-1] == n and np.all(pre == 0)
    # a spill that would reach two superblocks ahead is refused
    cmax = np.arange(100)
    cmax[0] = 60            # superblock [0, k) must stop by column 63
    cmax[70] = 99
    rc, r0s, spans, pre = _plan(pkg, cmax, 64)
    assert rc in (0, -1)
    if rc == 0:
        assert np.all(pre[1:] <= np.diff(r0s)[1:])


@pytest.mark.parametrize("P", [2, 3, 4])
def test_symsell_plan_row_distribution(pkg, P):
    """Rank blocks of a banded operator (as arpack_hip_dist_create hands them to
    the symmetric layout): each block's plan with spill_in = the previous
    rank's reach and spill_out = its own; local windows + the forward spill
    added into the next rank's first rows reproduce the global A @ x."""
    n, B = 6000, 300
    rp, col, val = M.banded_sym(n, 1234, B, 9)
    x = np.random.default_rng(9).standard_normal(n)
    yref = M.to_scipy(rp, col, val) @ x
    scale = M.to_scipy(rp, col, np.abs(val)) @ np.abs(x)
    bounds = [(q * n // P, (q + 1) * n // P) for q in range(P)]
    reach = []
    for a, b in bounds:   # how far each block's upper rows reach past its end
        c = col[rp[a]:rp[b]]
        reach.append(max(0, int(c.max()) - (b - 1)))
    y = np.zeros(n)
    carry = None
    for q, (a, b) in enumerate(bounds):
        lrp = rp[a:b + 1] - rp[a]
        lcol = col[rp[a]:rp[b]].astype(np.int64) - a          # diagonal at local index
        lval = val[rp[a]:rp[b]]
        sin = reach[q - 1] if q > 0 else 0
        sout = reach[q] if q < P - 1 else 0
        rc, r0s, spans, pre = _plan(pkg, _upper_cmax(lrp, lcol), 2048, sin, sout)
        assert rc == 0 and pre[0] == sin
        m = b - a
        yl = np.zeros(m + sout)
        for i in range(m):    # upper rows of the block, transposed terms included
            for k in range(lrp[i], lrp[i + 1]):
                j = lcol[k]
                if j < i:
                    continue
                yl[i] += lval[k] * x[a + j]
                if j != i:
                    yl[j] += lval[k] * x[a + i]
        if carry is not None:
            yl[:len(carry)] += carry
        y[a:b] = yl[:m]
        carry = yl[m:]
        assert spans[-1] - (r0s[-1] - r0s[-2]) <= sout
    assert np.all(np.abs(y - yref) <= 1e-13 * scale)


@pytest.mark.parametrize("P", [2, 3, 4])
def test_symsell_spill_free_row_distribution(pkg, P):
    """The spill-free distributed form (spmv_sym.hip k_ssell_combine_lg, agreed
    at arpack_hip_csr_set_symmetric): no spill crosses ranks; each block's
    leading pre[0] rows add their lower ghost terms -- the entries of the rank's
    own full rows whose columns lie before the block, over the low halo of x --
    and the rank's own spill past its end is dropped.  Its condition: every row
    with such an entry lies inside pre[0] (the rows the previous rank reaches);
    then the blocks reproduce the global A @ x."""
    n, B = 6000, 300
    rp, col, val = M.banded_sym(n, 1234, B, 9)
    x = np.random.default_rng(9).standard_normal(n)
    yref = M.to_scipy(rp, col, val) @ x
    scale = M.to_scipy(rp, col, np.abs(val)) @ np.abs(x)
    bounds = [(q * n // P, (q + 1) * n // P) for q in range(P)]
    reach = []
    for a, b in bounds:
        c = col[rp[a]:rp[b]]
        reach.append(max(0, int(c.max()) - (b - 1)))
    y = np.zeros(n)
    for q, (a, b) in enumerate(bounds):
        lrp = rp[a:b + 1] - rp[a]
        lcol = col[rp[a]:rp[b]].astype(np.int64) - a
        lval = val[rp[a]:rp[b]]
        sin = reach[q - 1] if q > 0 else 0
        sout = reach[q] if q < P - 1 else 0
        rc, r0s, spans, pre = _plan(pkg, _upper_cmax(lrp, lcol), 2048, sin, sout)
        assert rc == 0 and pre[0] == sin
        m = b - a
        rows = np.repeat(np.arange(m), np.diff(lrp))
        low = lcol < 0
        lg_rows = int(rows[low].max()) + 1 if low.any() else 0
        assert lg_rows <= pre[0]                   # the form's agreement condition
        yl = np.zeros(m + sout)
        for i in range(m):    # upper rows of the block, transposed terms included
            for k in range(lrp[i], lrp[i + 1]):
                j = lcol[k]
                if j < i:
                    continue
                yl[i] += lval[k] * x[a + j]
                if j != i:
                    yl[j] += lval[k] * x[a + i]
        for i in range(pre[0]):   # the leading rows' lower ghost terms, CSR order
            s = 0.0
            for k in range(lrp[i], lrp[i + 1]):
                if lcol[k] < 0:
                    s += lval[k] * x[a + lcol[k]]
            yl[i] += s
        y[a:b] = yl[:m]           # yl[m:] (the spill) is not sent
    assert np.all(np.abs(y - yref) <= 1e-13 * scale)


@pytest.mark.parametrize("P", [1, 2, 4, 8])
def test_symsell_plan_bench_sizes(pkg, P):
    """The bench's row blocks (n = 1e7 over P ranks, band 4096): every rank gets a
    plan whose superblock count is a multiple of 256 (one chain per CU, the
    chained k_csr_ssell), with the neighbours' spills at both ends."""
    n, B = 10_000_000, 4096
    for q in range(P):
        a, b = q * n // P, (q + 1) * n // P
        cmax = np.minimum(np.arange(a, b) + B - 1, n - 1) - a
        sin = B - 1 if q > 0 else 0
        sout = B - 1 if q < P - 1 else 0
        rc, r0s, spans, pre = _plan(pkg, cmax, 10240, sin, sout)
        assert rc == 0 and r0s[-1] == b - a
        assert len(spans) % 256 == 0
        assert pre[0] == sin and spans[-1] - (r0s[-1] - r0s[-2]) <= sout


@pytest.mark.parametrize("n", [1_250_000, 10_000_000])
def test_symsell_plan_light_first_superblock(pkg, n):
    """Workgroup 0 walks chain 0 and then runs the step's deferred finalize, so
    the plan gives chain 0's first superblock ~8% of a chain fewer rows (the
    finalize overlaps the other chains); the superblock count stays a multiple
    of the 256 CUs, the others stay balanced to one row, and inside chains
    (n = 1e7: 7 a chain) every window still satisfies the in-LDS shift's
    span <= 2R."""
    cm = np.minimum(np.arange(n) + 4095, n - 1).astype(np.int64)
    rc, r0s, spans, pre = _plan(pkg, cm, 10240)
    assert rc == 0 and len(spans) % 256 == 0
    R = np.diff(r0s)
    chain = len(spans) // 256
    assert R[1:].max() - R[1:].min() <= 1
    light = R[1] - R[0]
    assert 0 < light <= 0.09 * R[1] * chain + 1
    assert abs(light - 0.08 * R[1] / chain) <= 0.01 * R[1] + 1
    if chain > 1:
        assert np.all(spans <= 2 * R)
