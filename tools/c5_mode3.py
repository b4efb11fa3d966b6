"""BASELINE config 5 as stated: znaupd in shift-invert mode 3 on the complex
random CSR operator (n = 5e5, ~100 nnz/row, diag += 100), sigma = 0, LM,
nev 10, ncv 40, OP = (A - sigma I)^{-1} by the device BiCGStab
(arpack_hip_znaupd_zshift; csrc/zsolve.hip), capped at --cycles restart cycles.

    python tools/c5_mode3.py [--cycles 4] [--rtol 1e-12]
prints one JSON line: restart cycles/s, OP applications (solves), BiCGStab
iterations a solve, and the solve's roofline (algorithmic bytes of an iteration
x iterations / the solves' hipEvent time).  Also the target of the rocprofv3
passes for the complex kernels (tools/profile_c5.sh).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import HBM_PEAK_GBS, load_pkg  # noqa: E402


def _capped(pkg, Z, cycles, rtol, sigma):
    S = pkg.ZShift(Z, sigma, rtol=rtol, maxit=200)
    s = pkg.ZRci(Z.n, 10, 40, "LM", 0.0, mode=3, mxiter=cycles)
    pkg.synchronize()
    t = time.perf_counter()
    ido = s.aupd_zshift(S)
    pkg.synchronize()
    return s, S, ido, time.perf_counter() - t


def run(pkg, cycles=4, rtol=1e-12, n=500_000, sigma=0j):
    Z = pkg.ZCSR.random(n, 100, 5, 100.0)
    # steady state: the same solve capped at one cycle, subtracted from the
    # capped run -- removes the workspace setup, the start vector and the
    # initial nev-step factorisation, which both runs share
    s1, S1, _, el1 = _capped(pkg, Z, 1, rtol, sigma)
    opx1, ms1, s1_cycles = int(s1.iparam[8]), S1.stats()["ms"], int(s1.iparam[2])
    del s1, S1
    s, S, ido, el = _capped(pkg, Z, cycles, rtol, sigma)
    st = S.stats()
    steady = None
    c1, ck = int(s1_cycles), int(s.iparam[2])  # iparam(3) on return: the cycles taken
    if ck > c1:
        dt = el - el1
        steady = dict(cycles="%d..%d" % (c1 + 1, ck), seconds=dt, cycles_per_s=(ck - c1) / dt,
                      opx=int(s.iparam[8]) - opx1,
                      solve_share=(st["ms"] - ms1) * 1e-3 / dt if dt > 0 else None)
    solve_s = st["ms"] * 1e-3
    by = st["bytes_per_iter"] * st["iters"]
    gbs = by / solve_s / 1e9 if solve_s > 0 else None
    return dict(
        n=n, nnz=Z.nnz, which="LM", nev=10, ncv=40, mode=3, sigma=[sigma.real, sigma.imag],
        rtol=rtol, ido=ido, info=int(s.info[0]), cycles=int(s.iparam[2]),
        opx=int(s.iparam[8]), seconds=el, iters_per_s_incl_setup=int(s.iparam[2]) / el,
        solves=st["solves"], bicgstab_iters_per_solve=st["iters"] / max(1, st["solves"]),
        ms_per_solve=st["ms"] / max(1, st["solves"]), solve_share_of_time=solve_s / el,
        failures=st["failures"], max_relres=st["max_relres"], steady_state=steady,
        solver_roofline=dict(bound="hbm", achieved=gbs, peak=HBM_PEAK_GBS, unit="GB/s",
                             frac=(gbs / HBM_PEAK_GBS) if gbs else None,
                             bytes_per_iter=st["bytes_per_iter"],
                             tile_form=Z.tile_info()[0], stored_entries=Z.tile_info()[1],
                             bytes_model="per BiCGStab iteration: two products over the "
                                         "column-sorted tiles -- packed (tile_form 3): 18 B a "
                                         "stored complex entry (16 B value + 2 B row / column-"
                                         "step code) + 4 B a 64-entry chunk, stored entries "
                                         "incl. fillers and padding; tile_form 2: 20 B an entry "
                                         "(16 B value + 4 B row | column) -- + 8 B rowptr + 16 B "
                                         "x a row, feeding v and t directly, and 19 complex "
                                         "n-vector passes of the fused updates (csrc/zsolve.hip "
                                         "zshift_iter_bytes)"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=4)
    ap.add_argument("--rtol", type=float, default=1e-12)
    a = ap.parse_args()
    print(json.dumps(run(load_pkg(), a.cycles, a.rtol)), flush=True)


if __name__ == "__main__":
    main()
