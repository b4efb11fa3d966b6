"""Cost model of a fixed-order (deterministic) symmetric-storage SpMV by edge
colouring: within one superblock of the NS operator, every
upper-triangle entry (i, c) adds to y_i (row part) and y_c (transposed part);
an "epoch" may hold each destination at most once, so the epochs are the colour
classes of a proper edge colouring of the superblock's graph and the sums are
ordered by epoch (barriers between epochs).  Prints the entries, the largest
vertex degree (the lower bound on epochs), the greedy colour count, the epoch
size spread and the padding to whole waves.

    python tools/sym_coloring.py [--n 30000] [--band 4096] [--r0 8192] [--rows 4097]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import matrices as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=30000)
ap.add_argument("--band", type=int, default=4096)
ap.add_argument("--per-row", type=int, default=25)
ap.add_argument("--r0", type=int, default=8192)
ap.add_argument("--rows", type=int, default=4097)
a = ap.parse_args()
rp, col, _ = M.banded_sym(a.n, 1234, a.band, a.per_row)
rows, cols = [], []
for i in range(a.r0, a.r0 + a.rows):
    c = col[rp[i]:rp[i + 1]]
    c = c[c >= i]
    rows += [i - a.r0] * len(c)
    cols += list(c - a.r0)
rows, cols = np.array(rows), np.array(cols)
nv = int(cols.max()) + 1
off = cols != rows
deg = np.bincount(rows, minlength=nv) + np.bincount(cols[off], minlength=nv)
used = [0] * nv
color = np.empty(len(rows), int)
for e in np.argsort(-(deg[rows] + deg[cols]), kind="stable"):
    u, v = rows[e], cols[e]
    m = used[u] | used[v]
    c = 0
    while (m >> c) & 1:
        c += 1
    color[e] = c
    used[u] |= 1 << c
    if v != u:
        used[v] |= 1 << c
cnt = np.bincount(color)
pad = sum((-k) % 64 for k in cnt)
print("superblock rows %d, entries %d (%.1f a row), window %d" % (a.rows, len(rows), len(rows) / a.rows, nv))
print("max vertex degree %d (mean %.1f over the rows): epochs >= %d" % (deg.max(), deg[:a.rows].mean(), deg.max()))
print("greedy colours (epochs) %d; epoch sizes min/mean/max %d / %.0f / %d" % (cnt.size, cnt.min(), cnt.mean(), cnt.max()))
print("padding to whole waves %.1f%%; bytes per entry 8 (value) + 4 (row, column) = 12 vs 10 today"
      % (100.0 * pad / len(rows)))
