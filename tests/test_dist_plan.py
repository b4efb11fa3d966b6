"""CPU: the row-block decomposition of the multi-GPU engine.

* arpack_hip_kit_halo_plan (the host half of arpack_hip_dist_create) against the
  halo sizes computed directly from the CSR column span of each block;
* the plan's semantics: assembling every rank's extended x from its neighbours'
  send slices reproduces the global SpMV exactly (the exchange that
  comm_halo performs with ncclSend/ncclRecv);
* partition_rows == PARPACK/TESTS/MPI/icb_parpack_c.c:60-77's balanced split.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import matrices as M


def _plan(pkg, tab, P, r):
    L = pkg.lib()
    L.arpack_hip_kit_halo_plan.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_double),
                                           C.POINTER(C.c_int64)]
    out = np.zeros(4, np.int64)
    t = np.ascontiguousarray(tab, np.float64)
    rc = L.arpack_hip_kit_halo_plan(P, r, t.ctypes.data_as(C.POINTER(C.c_double)),
                                    out.ctypes.data_as(C.POINTER(C.c_int64)))
    return rc, out


def _table(rp, col, bounds):
    tab = []
    for r0, r1 in bounds:
        c = col[rp[r0]:rp[r1]]
        tab += [r0, r1 - r0, c.min() if len(c) else r0, c.max() if len(c) else r0]
    return np.array(tab, np.float64)


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_halo_plan_and_exchange_reproduce_global_spmv(pkg, P):
    n = 6000
    rp, col, val = M.banded_sym(n, 1234, 300, 9)
    A = M.to_scipy(rp, col, val)
    x = np.random.default_rng(P).standard_normal(n)
    y_ref = A @ x
    bounds = [pkg.partition_rows(n, P, r) for r in range(P)]
    tab = _table(rp, col, bounds)
    plans = []
    for r in range(P):
        rc, p = _plan(pkg, tab, P, r)
        assert rc == 0
        r0, r1 = bounds[r]
        c = col[rp[r0]:rp[r1]]
        assert p[0] == max(0, r0 - c.min()) and p[1] == max(0, c.max() - (r1 - 1))
        plans.append(p)
    for r in range(P):  # what r sends to r-1 is exactly what r-1 expects from r
        if r > 0:
            assert plans[r][2] == plans[r - 1][1]
        if r < P - 1:
            assert plans[r][3] == plans[r + 1][0]
    for r in range(P):  # assemble x_ext from the neighbours' send slices, local SpMV
        r0, r1 = bounds[r]
        hlo, hhi = plans[r][0], plans[r][1]
        parts = []
        if hlo:
            q0, q1 = bounds[r - 1]
            parts.append(x[q0:q1][(q1 - q0) - plans[r - 1][3]:])
        parts.append(x[r0:r1])
        if hhi:
            q0, q1 = bounds[r + 1]
            parts.append(x[q0:q1][:plans[r + 1][2]])
        xe = np.concatenate(parts)
        assert len(xe) == hlo + (r1 - r0) + hhi
        lrp = rp[r0:r1 + 1] - rp[r0]
        lcol = col[rp[r0]:rp[r1]] - (r0 - hlo)
        lval = val[rp[r0]:rp[r1]]
        y = np.array([lval[lrp[i]:lrp[i + 1]] @ xe[lcol[lrp[i]:lrp[i + 1]]]
                      for i in range(r1 - r0)])
        np.testing.assert_allclose(y, y_ref[r0:r1], rtol=1e-13, atol=1e-12)


def test_halo_plan_rejects_bad_layouts(pkg):
    # non-contiguous blocks
    tab = np.array([0, 10, 0, 12, 11, 10, 9, 20], np.float64)
    assert _plan(pkg, tab, 2, 0)[0] == -3
    # halo wider than the neighbour's block
    tab = np.array([0, 10, 0, 25, 10, 10, 8, 19, 20, 10, 18, 29], np.float64)
    assert _plan(pkg, tab, 3, 0)[0] == -4
    # first rank referencing columns below 0 / last above n-1
    tab = np.array([0, 10, -1, 12, 10, 10, 8, 19], np.float64)
    assert _plan(pkg, tab, 2, 1)[0] == -4
    assert _plan(pkg, tab, 2, 5)[0] == -1


def test_partition_rows_balanced(pkg):
    for n, P in [(10, 3), (10_000_000, 8), (7, 8), (1000, 1)]:
        b = [pkg.partition_rows(n, P, r) for r in range(P)]
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[i][1] == b[i + 1][0] for i in range(P - 1))
        sizes = [e - s for s, e in b]
        assert max(sizes) - min(sizes) <= 1
