"""numpy restatement of the synthetic operators of arpack-ng_amd/csrc/csr.hip.

TEST INFRASTRUCTURE ONLY (same rules as oracle/ref.py).  Used to feed the
reference (oracle/_ref) and the CPU baseline the very same matrices the GPU
generators build in HBM.  All values lie on power-of-two grids, so the CSR
arrays produced here and on the device are bit-identical (checked by
tests/test_matrices.py on the GPU).

  laplace2d(m, scale)   5-pt Laplacian on an m x m grid; scale=(m+1)^2 gives the
                        operator of EXAMPLES/SIMPLE/dssimp.f (av/tv, :484-538)
  laplace3d(m, scale)   7-pt Laplacian on m^3
  banded_sym(n, seed, B, per_row, r0, r1)
                        north-star symmetric CSR (SURVEY.md §8d "NS")
  diag(n)               diag(1..n) of TESTS/icb_arpack_c.c:25-27
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def _mix32(x):
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def _pair_hash(seedmix, a, d):
    t = (_mix32(np.asarray(a, np.uint64) ^ seedmix) + np.asarray(d, np.uint64) * np.uint64(0x9E3779B9)) & M32
    return _mix32(t)


def _offdiag_value(h):
    k = (_mix32(h ^ np.uint64(0x68E31DA4)) >> np.uint64(20)) + np.uint64(1)
    return -(k.astype(np.float64)) * 2.0 ** -12


def _diag_shift(seed, i):
    s2 = _mix32(np.uint64(seed) ^ np.uint64(0x5BD1E995))
    return (_mix32(np.asarray(i, np.uint64) ^ s2) >> np.uint64(20)).astype(np.float64) * 2.0 ** -8


def banded_sym(n, seed=1234, B=4096, per_row=25, r0=0, r1=None):
    """Rows [r0, r1) of the north-star matrix (global column indices)."""
    r1 = n if r1 is None else r1
    sm = _mix32(np.uint64(seed))
    rows = np.arange(r0, r1, dtype=np.int64)
    cols_l, vals_l, rows_l = [], [], []
    # lower part: pair (i-d, d), upper part: pair (i, d)
    for d in range(1, B):
        lo = rows - d
        ok = lo >= 0
        h = _pair_hash(sm, np.where(ok, lo, 0), d)
        ok &= (h >> np.uint64(20)) < np.uint64(per_row)
        rows_l.append(rows[ok]); cols_l.append(lo[ok]); vals_l.append(_offdiag_value(h[ok]))
        hi = rows + d
        ok = hi < n
        h = _pair_hash(sm, rows, d)
        ok &= (h >> np.uint64(20)) < np.uint64(per_row)
        rows_l.append(rows[ok]); cols_l.append(hi[ok]); vals_l.append(_offdiag_value(h[ok]))
    r = np.concatenate(rows_l) if rows_l else np.zeros(0, np.int64)
    c = np.concatenate(cols_l) if cols_l else np.zeros(0, np.int64)
    v = np.concatenate(vals_l) if vals_l else np.zeros(0)
    # diagonal: -sum(offdiag) + U[0,16) on a 2^-8 grid (exact in any order)
    offsum = np.zeros(r1 - r0)
    np.add.at(offsum, r - r0, v)
    dg = -offsum + _diag_shift(seed, rows)
    r = np.concatenate([r, rows]); c = np.concatenate([c, rows]); v = np.concatenate([v, dg])
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    counts = np.bincount(r - r0, minlength=r1 - r0)
    rowptr = np.zeros(r1 - r0 + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr, c.astype(np.int32), v


def laplace(m, dim=2, scale=1.0, disorder=0.0, seed=0):
    n = m ** dim
    i = np.arange(n, dtype=np.int64)
    x = i % m
    y = (i // m) % m
    z = i // (m * m) if dim == 3 else np.zeros_like(i)
    entries = []
    off = -1.0 * scale
    dg = (4.0 if dim == 2 else 6.0) * scale
    if dim == 3:
        entries.append((z > 0, i - m * m, off))
    dgv = np.full(n, dg)
    if disorder != 0.0:
        s2 = _mix32(np.uint64(seed) ^ np.uint64(0x2545F491))
        u = (_mix32(i.astype(np.uint64) ^ s2) >> np.uint64(20)).astype(np.float64) * 2.0 ** -12
        dgv = dg + disorder * u
    entries += [(y > 0, i - m, off), (x > 0, i - 1, off), (np.ones(n, bool), i, dgv),
                (x < m - 1, i + 1, off), (y < m - 1, i + m, off)]
    if dim == 3:
        entries.append((z < m - 1, i + m * m, off))
    r = np.concatenate([i[ok] for ok, _, _ in entries])
    c = np.concatenate([j[ok] for ok, j, _ in entries])
    v = np.concatenate([np.asarray(val)[ok] if np.ndim(val) else np.full(int(ok.sum()), val)
                        for ok, _, val in entries])
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=n), out=rowptr[1:])
    return rowptr, c.astype(np.int32), v


def convdiff2d(m, rho):
    """-Lap u + rho du/dx on an m x m grid, coefficients as
    EXAMPLES/NONSYM/dndrv1.f:425,458-462 compute them (device twin:
    arpack_hip_gen_convdiff2d)."""
    n = m * m
    h = 1.0 / (m + 1)
    h2 = h * h
    dd = 4.0 / h2
    dl = -1.0 / h2 - 0.5 * rho / h
    du = -1.0 / h2 + 0.5 * rho / h
    offy = -1.0 / (1.0 / float((m + 1) * (m + 1)))
    i = np.arange(n, dtype=np.int64)
    x = i % m
    y = i // m
    entries = [(y > 0, i - m, offy), (x > 0, i - 1, dl), (np.ones(n, bool), i, dd),
               (x < m - 1, i + 1, du), (y < m - 1, i + m, offy)]
    r = np.concatenate([i[ok] for ok, _, _ in entries])
    c = np.concatenate([j[ok] for ok, j, _ in entries])
    v = np.concatenate([np.full(int(ok.sum()), val) for ok, _, val in entries])
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=n), out=rowptr[1:])
    return rowptr, c.astype(np.int32), v


def zrandom(n, per_row=100, seed=5, dshift=100.0):
    """Complex random CSR of BASELINE config 5, the numpy twin
    of arpack_hip_gen_zrandom: row i draws per_row columns hash(seed,i,k) mod n
    with values U(-1,1)+iU(-1,1) on a 2^-10 grid (duplicates summed -- exact),
    plus dshift on the diagonal."""
    sm = _mix32(np.uint64(seed))
    i = np.repeat(np.arange(n, dtype=np.uint64), per_row)
    k = np.tile(np.arange(per_row, dtype=np.uint64), n)
    h = _mix32((_mix32(i ^ sm) + k * np.uint64(0x9E3779B9)) & M32)
    col = (h % np.uint64(n)).astype(np.int64)
    re = (_mix32(h ^ np.uint64(0x68E31DA4)) >> np.uint64(21)).astype(np.float64) * 2.0 ** -10 - 1.0
    im = (_mix32(h ^ np.uint64(0x1B873593)) >> np.uint64(21)).astype(np.float64) * 2.0 ** -10 - 1.0
    rows = i.astype(np.int64)
    rows = np.concatenate([rows, np.arange(n, dtype=np.int64)])
    col = np.concatenate([col, np.arange(n, dtype=np.int64)])
    val = np.concatenate([re + 1j * im, np.full(n, dshift + 0j)])
    key = rows * n + col
    uk, inv = np.unique(key, return_inverse=True)
    v = np.zeros(len(uk), np.complex128)
    np.add.at(v, inv, val)
    r, c = uk // n, uk % n
    rowptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=n), out=rowptr[1:])
    return rowptr, c.astype(np.int32), v


def zdiag_icb(n=1000):
    """TESTS/icb_arpack_c.c:93-96 zMatVec: y_i = (i+1)(1+i) x_i, as CSR."""
    i = np.arange(n, dtype=np.int64)
    return np.arange(n + 1, dtype=np.int64), i.astype(np.int32), (i + 1.0) * (1 + 1j)


def laplace2d(m, scale=1.0):
    return laplace(m, 2, scale)


def laplace3d(m, scale=1.0):
    return laplace(m, 3, scale)


def anderson(m, dim=3, disorder=16.0, seed=1234):
    return laplace(m, dim, 1.0, disorder, seed)


def diag(n):
    rowptr = np.arange(n + 1, dtype=np.int64)
    return rowptr, np.arange(n, dtype=np.int32), np.arange(1, n + 1, dtype=np.float64)


def to_scipy(rowptr, col, val, ncols=None):
    import scipy.sparse as sp
    n = len(rowptr) - 1
    return sp.csr_matrix((val, col, rowptr), shape=(n, ncols or n))


def dlarnv_uniform(n, iseed=(1, 3, 5, 7)):
    """LAPACK dlarnv(idist=2) (dlaruv's 48-bit MCG, multiplier 33952834046453):
    x_m = seed*a^m mod 2^48, value 2*x/2^48 - 1.  Returns (values, new_iseed).
    Pinned against the image's LAPACK by tests/golden/g7_dlarnv.npz."""
    a = 33952834046453
    mask = (1 << 48) - 1
    s = (iseed[0] << 36) | (iseed[1] << 24) | (iseed[2] << 12) | iseed[3]
    out = np.empty(n)
    # chunked vectorised powers: x_m = s * a^m
    pw = [1]
    for _ in range(64):
        pw.append((pw[-1] * a) & mask)
    k = 0
    while k < n:
        c = min(64, n - k)
        xs = [(s * pw[t]) & mask for t in range(1, c + 1)]
        out[k:k + c] = 2.0 * (np.array(xs, dtype=np.float64) * 2.0 ** -48) - 1.0
        s = xs[-1]
        k += c
    return out, ((s >> 36) & 4095, (s >> 24) & 4095, (s >> 12) & 4095, s & 4095)
