"""Time the full-storage SELL SpMV variants (arpack_hip_csr_set_kernel(11, u))
on the bench operator; each variant's y is checked bitwise against the default.

    python tools/spmv_full_time.py [--n N] [--reps R]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    pkg = load_pkg()
    A = pkg.CSR.banded_sym(a.n, 1234, 4096, 25)
    x = pkg.DeviceBuffer(a.n)
    x.write(np.random.default_rng(1).standard_normal(a.n))
    y0 = pkg.DeviceBuffer(a.n)
    y1 = pkg.DeviceBuffer(a.n)
    A.matvec_device(x.at(0), y0.at(0))
    ref = y0.numpy()
    out = {}
    for u in (4, 9, 10, 11, 4, 9):
        A.set_kernel(11, u)
        ms = A.time_spmv(a.reps)
        A.matvec_device(x.at(0), y1.at(0))
        out.setdefault("u%d_ms" % u, []).append(round(ms, 4))
        out["u%d_bitwise" % u] = bool(np.array_equal(y1.numpy(), ref))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
