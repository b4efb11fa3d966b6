"""Where the north star's time to converge goes: the same solve as bench.py's
TTC (NS operator, n = 1e7, LA, nev 10, ncv 30, tol 1e-6, dlarnv 1,3,5,7 start)
split into the first aupd call (engine setup + getv0 + the initial nev-step
factorisation) and the restart cycles, each bracketed by device syncs.
    python tools/ttc_breakdown.py [--n N]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
args = ap.parse_args()
pkg = bench.load_pkg()
n = args.n
A = pkg.CSR.banded_sym(n, 1234, 4096, 25, 0, n)
A.set_symmetric(True)
for rep in range(2):
    iseed = np.array([1, 3, 5, 7], np.int32)
    v0 = np.empty(n, np.float64)
    pkg.lib().arpack_hip_kit_dlarnv(iseed.ctypes.data_as(pkg.C.POINTER(pkg.C.c_int)), n,
                                    v0.ctypes.data_as(pkg.C.POINTER(pkg.C.c_double)))
    s = pkg.SymRci(n, 10, 30, "LA", 1e-6, mxiter=300, device=True, v0=v0)
    pkg.synchronize()
    t0 = time.perf_counter()
    s.aupd_cycles(A, 0)
    pkg.synchronize()
    t1 = time.perf_counter()
    nop0 = pkg.stats()["nopx"]
    s.aupd_cycles(A, -1)
    pkg.synchronize()
    t2 = time.perf_counter()
    print(f"rep {rep}: first call (setup + getv0 + {nop0} OP*x) {1e3 * (t1 - t0):.1f} ms, "
          f"cycles {int(s.iparam[2])} ({int(s.iparam[8]) - nop0} OP*x) {1e3 * (t2 - t1):.1f} ms, "
          f"total {1e3 * (t2 - t0):.1f} ms", flush=True)
    del s
