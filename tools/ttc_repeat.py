"""Run-to-run spread of the north star's time-to-converge solve (the bench's TTC
case: NS operator n = 1e7, LA, nev 10, ncv 30, tol 1e-6, start vector = the
reference's first dlarnv draw), repeated R times in one process with each SpMV
storage:

  sym   the bench default (since round 6): upper-triangle SpMV with the
        transposed terms as 64-bit fixed-point sums -- bitwise reproducible;
  sym_fp64  the same kernel with the LDS fp64 accumulator: the transposed terms
        land in wave-schedule order -- y reproducible to rounding, not bitwise;
  full  SELL-64 full storage, bitwise SciPy's csr_matvec: bitwise reproducible.

Reported per storage: restart cycles and OP*x of every run, the largest spread
of each Ritz value across the runs (relative), and, for sym, the largest
distance to the full-storage Ritz values.  One JSON line.

    python tools/ttc_repeat.py [--repeats 8]
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
    ap.add_argument("--repeats", type=int, default=8)
    ap.add_argument("--n", type=int, default=10_000_000)
    a = ap.parse_args()
    pkg = load_pkg()
    n = a.n
    A = pkg.CSR.banded_sym(n, 1234, 4096, 25, 0, n)
    iseed = np.array([1, 3, 5, 7], np.int32)
    v0 = np.empty(n, np.float64)
    pkg.lib().arpack_hip_kit_dlarnv(iseed.ctypes.data_as(pkg.C.POINTER(pkg.C.c_int)), n,
                                    v0.ctypes.data_as(pkg.C.POINTER(pkg.C.c_double)))
    out = {}
    ref = None
    for storage in ("full", "sym", "sym_fp64"):
        A.set_symmetric(storage != "full")
        if storage != "full":
            A.set_sym_accumulator("fp64" if storage == "sym_fp64" else "fixed")
        runs, ds = [], []
        for _ in range(a.repeats):
            s = pkg.SymRci(n, 10, 30, "LA", 1e-6, mxiter=300, device=True, v0=v0)
            pkg.synchronize()
            t = time.perf_counter()
            s.aupd_cycles(A, -1)
            pkg.synchronize()
            secs = time.perf_counter() - t
            d, _, nconv = s.eupd(rvec=False)
            runs.append(dict(cycles=int(s.iparam[2]), opx=int(s.iparam[8]), nconv=nconv,
                             seconds=round(secs, 4)))
            ds.append(np.sort(d))
            del s
        D = np.array(ds)
        spread = float(np.max((D.max(0) - D.min(0)) / np.abs(D).max(0)))
        rec = dict(runs=runs, ritz_spread_rel=spread, spmv_form=A.sym_form,
                   cycles_distinct=sorted({r["cycles"] for r in runs}),
                   bitwise_identical=bool(np.all(D.view(np.int64) == D[0].view(np.int64))),
                   seconds_median=float(np.median([r["seconds"] for r in runs])))
        if storage == "full":
            ref = D[0]
        else:
            rec["max_rel_diff_to_full"] = float(np.max(np.abs(D - ref) / np.abs(ref)))
        out[storage] = rec
        print(json.dumps({storage: rec}), file=sys.stderr, flush=True)
    out["ritz_full"] = [float(x) for x in ref]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
