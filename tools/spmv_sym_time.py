"""Time the full-storage SELL SpMV against the symmetric-storage kernel on the
bench operator (NS, n = 1e7) and report their agreement.

    python tools/spmv_sym_time.py [--n N] [--reps R]
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
    ap.add_argument("--variants", type=int, nargs="*", default=[3, 4, 5, 6, 7])
    a = ap.parse_args()
    pkg = load_pkg()
    A = pkg.CSR.banded_sym(a.n, 1234, 4096, 25)
    out = {"n": a.n, "nnz": A.nnz}
    x = pkg.DeviceBuffer(a.n)
    x.write(np.random.default_rng(1).standard_normal(a.n))
    y1 = pkg.DeviceBuffer(a.n)
    y2 = pkg.DeviceBuffer(a.n)
    out["full_ms"] = A.time_spmv(a.reps)
    A.matvec_device(x.at(0), y1.at(0))
    A.set_symmetric(True)
    out["sym_ms"] = A.time_spmv(a.reps)
    A.matvec_device(x.at(0), y2.at(0))
    for i, v in enumerate(a.variants):
        A.set_kernel(12, v)
        key = "sym_v%d_ms" % v if "sym_v%d_ms" % v not in out else "sym_v%d_ms_%d" % (v, i)
        out[key] = A.time_spmv(a.reps)
        A.matvec_device(x.at(0), y2.at(0))
        d = np.abs(y1.numpy() - y2.numpy())
        out["sym_v%d_maxrel" % v] = float((d / np.maximum(np.abs(y1.numpy()), 1e-300)).max())
    A.set_kernel(12, 0)
    out["sym_ms_again"] = A.time_spmv(a.reps)
    A.matvec_device(x.at(0), y2.at(0))
    d = np.abs(y1.numpy() - y2.numpy())
    out["max_abs_diff"] = float(d.max())
    out["max_rel_diff"] = float((d / np.maximum(np.abs(y1.numpy()), 1e-300)).max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
