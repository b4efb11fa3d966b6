"""Time the complex CSR SpMV (arpack_hip_zcsr_spmv) on the BASELINE config-5
operator (n = 5e5, 100 entries/row) and check it against SciPy.

    AHIP_ZCSR_G=16 python tools/zspmv_time.py [--n N] [--reps R]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500_000)
    ap.add_argument("--per-row", type=int, default=100)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    pkg = load_pkg()
    Z = pkg.ZCSR.random(a.n, a.per_row, 5, 100.0)
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(a.n) + 1j * rng.standard_normal(a.n)).astype(np.complex128)
    xd = pkg.DeviceBuffer.from_numpy(x.view(np.float64))
    yd = pkg.DeviceBuffer(2 * a.n)
    L = pkg.lib()
    L.arpack_hip_zcsr_spmv(Z.h, xd.ptr, yd.ptr)
    pkg.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        L.arpack_hip_zcsr_spmv(Z.h, xd.ptr, yd.ptr)
    pkg.synchronize()
    ms = 1e3 * (time.perf_counter() - t) / a.reps
    y = yd.numpy().view(np.complex128)
    import scipy.sparse as sp
    rp, col, val = Z.download()
    ref = sp.csr_matrix((val, col, rp), shape=(a.n, a.n)) @ x
    err = np.abs(y - ref).max() / np.abs(ref).max()
    algo = Z.nnz * 20 + (a.n + 1) * 8 + a.n * 32  # val + col + rowptr + x + y
    print(json.dumps(dict(G=os.environ.get("AHIP_ZCSR_G", "auto"), n=a.n, nnz=Z.nnz, ms=ms,
                          algo_gbs=algo / (ms * 1e-3) / 1e9, max_rel_err=err)), flush=True)


if __name__ == "__main__":
    main()
