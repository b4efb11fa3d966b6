"""Isolated SpMV times on the n = 10^6 BASELINE operators (configs 2 and 3):
the default kernel and the full-storage SELL unrolls (arpack_hip_csr_set_kernel(11, u)),
each variant's y checked bitwise against the default.

    python tools/spmv_small.py [--reps R]
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
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    pkg = load_pkg()
    out = {}
    for name, make in (("C2_lap2d", lambda: pkg.CSR.laplace2d(1000)),
                       ("C3_convdiff", lambda: pkg.CSR.convdiff2d(1000, 10.0))):
        A = make()
        n = A.n
        x = pkg.DeviceBuffer(n)
        x.write(np.random.default_rng(1).standard_normal(n))
        y0, y1 = pkg.DeviceBuffer(n), pkg.DeviceBuffer(n)
        A.matvec_device(x.at(0), y0.at(0))
        ref = y0.numpy()
        rec = {"default_ms": round(A.time_spmv(a.reps), 4)}
        for u in (4, 8, 2, 3, 6, 9, 10, 11, 5, 7):
            A.set_kernel(11, u)
            rec["u%d_ms" % u] = round(A.time_spmv(a.reps), 4)
            A.matvec_device(x.at(0), y1.at(0))
            rec["u%d_bitwise" % u] = bool(np.array_equal(y1.numpy(), ref))
        out[name] = rec
        del A
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
