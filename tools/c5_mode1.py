"""Config 5's operator in mode 1 (OP = A): the complex Arnoldi engine alone.

    python tools/c5_mode1.py [--cycles 8] [--reps 3]
prints one JSON line: restart cycles/s of capped solves from the same start
(the first one warms the kernels up and is not counted), Ritz values of the
last solve, and the cycles/OP*x counts -- a same-box A/B of two builds runs it
under ARPACK_HIP_LIB=<other build>.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import load_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    pkg = load_pkg()
    n = 500_000
    Z = pkg.ZCSR.random(n, 100, 5, 100.0)
    times, cyc, opx = [], None, None
    for r in range(args.reps + 1):
        s = pkg.ZRci(n, 10, 40, "LM", 0.0, mxiter=args.cycles)
        pkg.synchronize()
        t = time.perf_counter()
        s.aupd_zcsr(Z)
        pkg.synchronize()
        if r:
            times.append(time.perf_counter() - t)
        cyc, opx = int(s.iparam[2]), int(s.iparam[8])
        del s
    best = min(times)
    print(json.dumps(dict(workload="C5 operator, znaupd mode 1, LM, nev 10, ncv 40", n=n,
                          cycles=cyc, opx=opx, seconds=times, cycles_per_s=cyc / best,
                          lib=os.environ.get("ARPACK_HIP_LIB", "default"))), flush=True)


if __name__ == "__main__":
    main()
