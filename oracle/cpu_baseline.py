"""CPU baseline for bench.py: the REAL reference (oracle/_ref: arpack-ng's
Fortran dsaupd_ + OpenBLAS) timed on the host cores, on a bounded sample of the
bench workload.  TEST/BENCH INFRASTRUCTURE ONLY — never the measured product.

Sample: the bench operator (identical CSR, generated on the GPU by the engine's
generator and copied to host memory) driven through the reference RCI loop with
a multithreaded OpenMP CSR SpMV as the user OP (oracle/csr_omp.c).  We time the
reference from the OP*x request that opens restart cycle 1 (request #12: one
getv0 request + nev0 = 10 initial Lanczos steps precede it) to the request that
opens cycle k + 1 (#12 + 20 k), i.e. exactly k implicit-restart cycles (np = 20
Lanczos steps + dseigt/dsgets/dsapps each), then stop; bench.py times the same
cycles of the same solve on the GPU.  --ttc adds the reference's full solve at
tol 1e-6 (the bench's time-to-converge case).  Run as a subprocess:

    python -m oracle.cpu_baseline --n 10000000 --threads 16 [--cycles 3] [--ttc]
prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def dlarnv_fast(n, iseed=(1, 3, 5, 7)):
    """Vectorised dlarnv(idist=2): x_m = s*a^m mod 2^48 (see oracle/matrices.py)."""
    import numpy as np
    a = 33952834046453
    mask = (1 << 48) - 1
    s = (iseed[0] << 36) | (iseed[1] << 24) | (iseed[2] << 12) | iseed[3]
    pw = [1]
    for _ in range(64):
        pw.append((pw[-1] * a) & mask)
    a64 = pw[64]
    nch = (n + 63) // 64
    starts = np.empty(nch, dtype=np.uint64)
    cur = s
    for c in range(nch):
        starts[c] = cur
        cur = (cur * a64) & mask
    tab = np.array(pw[1:65], dtype=np.uint64)
    m24 = np.uint64((1 << 24) - 1)
    s0 = starts[:, None] & m24
    s1 = starts[:, None] >> np.uint64(24)
    t0 = tab[None, :] & m24
    t1 = tab[None, :] >> np.uint64(24)
    lo = s0 * t0
    mid = ((s1 * t0 + s0 * t1) & m24) << np.uint64(24)
    x = (lo + mid) & np.uint64(mask)
    return (2.0 * (x.reshape(-1)[:n].astype(np.float64) * 2.0 ** -48) - 1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--bandwidth", type=int, default=4096)
    ap.add_argument("--per-row", type=int, default=25)
    ap.add_argument("--lap3d", type=int, default=0,
                    help="m > 0: the bench's lap3d workload (BASELINE config 4, the m^3 7-pt "
                         "Laplacian) in place of the banded operator; --n is m^3")
    ap.add_argument("--nev", type=int, default=10)
    ap.add_argument("--ncv", type=int, default=30)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--cycles", type=int, default=3,
                    help="restart cycles 1..k timed (np = ncv - nev Lanczos steps each)")
    ap.add_argument("--ttc", action="store_true",
                    help="also time the reference's full solve at --ttc-tol (time to converge)")
    ap.add_argument("--ttc-tol", type=float, default=1e-6)
    args = ap.parse_args()
    os.environ["OPENBLAS_NUM_THREADS"] = str(args.threads)
    os.environ["OMP_NUM_THREADS"] = str(args.threads)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import ctypes as C
    import importlib.util

    import numpy as np

    from oracle import ref

    d = os.path.join(root, "arpack-ng_amd")
    spec = importlib.util.spec_from_file_location("arpack_ng_amd", os.path.join(d, "__init__.py"),
                                                  submodule_search_locations=[d])
    pkg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pkg)
    t = time.time()
    if args.lap3d > 0:
        args.n = args.lap3d ** 3
        A = pkg.CSR.laplace3d(args.lap3d)
    else:
        A = pkg.CSR.banded_sym(args.n, args.seed, args.bandwidth, args.per_row)
    rowptr, col, val = A.download()
    del A
    t_gen = time.time() - t
    op = ref.csr_matvec(rowptr, col, val, nthreads=args.threads)
    n, nev, ncv = args.n, args.nev, args.ncv
    L = ref.lib()
    ido = np.zeros(1, np.int32)
    info = np.ones(1, np.int32)
    resid = dlarnv_fast(n)
    v = np.zeros(n * ncv)
    iparam = np.zeros(11, np.int32)
    ipntr = np.zeros(11, np.int32)
    iparam[0], iparam[2], iparam[6] = 1, 300, 1
    workd = np.zeros(3 * n)
    lworkl = ncv * ncv + 8 * ncv
    workl = np.zeros(lworkl)
    tol = C.c_double(0.0)
    P = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    nreq = 0
    stamps = {}
    np_ = ncv - nev
    # request #1 is getv0's, #2..#(nev+1) the initial factorisation, then cycle c
    # (np = ncv - nev steps while no Ritz value has converged, as in the GPU's
    # verified count of the same solve) opens at request 2 + nev + (c - 1) np
    opens = [2 + nev + c * np_ for c in range(args.cycles + 1)]
    t_start = time.time()
    while True:
        L.dsaupd_(P(ido), b"I", C.byref(C.c_int(n)), b"LA", C.byref(C.c_int(nev)), C.byref(tol),
                  P(resid), C.byref(C.c_int(ncv)), P(v), C.byref(C.c_int(n)), P(iparam),
                  P(ipntr), P(workd), P(workl), C.byref(C.c_int(lworkl)), P(info),
                  C.c_size_t(1), C.c_size_t(2))
        if ido[0] not in (-1, 1):
            break
        nreq += 1
        stamps[nreq] = time.time()
        if nreq == opens[-1]:  # the request opening cycle k + 1
            break
        x = workd[ipntr[0] - 1: ipntr[0] - 1 + n]
        workd[ipntr[1] - 1: ipntr[1] - 1 + n] = op(x)
    per_cycle = [stamps[opens[c + 1]] - stamps[opens[c]] for c in range(args.cycles)]
    cycle_s = sum(per_cycle) / len(per_cycle)
    out = dict(
        cycle_s=cycle_s, iters_per_s=1.0 / cycle_s, lanczos_steps_per_s=np_ / cycle_s,
        per_cycle_s=per_cycle, cycles="1..%d" % args.cycles, threads=args.threads,
        setup_s=stamps[opens[0]] - t_start, gen_download_s=t_gen, nnz=int(len(col)), n=n,
        kind="reference",
        sample=f"restart cycles 1..{args.cycles} (np={np_} Lanczos steps + dsapps each) of the "
               f"bench workload's ({'lap3d m=%d' % args.lap3d if args.lap3d else 'NS'}) tol=eps solve from dlarnv(1,3,5,7), reference Fortran dsaupd_ "
               f"+ OpenBLAS, OpenMP CSR OP, {args.threads} threads")
    del v, workd, workl
    if args.ttc:
        t = time.time()
        r = ref.dsaupd_solve(lambda x, *_: op(x), n, nev, ncv, "LA", args.ttc_tol,
                             v0=dlarnv_fast(n), mxiter=300, rvec=False)
        out["time_to_converge"] = dict(seconds=time.time() - t, iters=int(r["iparam"][2]),
                                       nopx=int(r["stats"]["nopx"]), info=int(r["info"]),
                                       nconv=int(r.get("nconv", 0)), tol=args.ttc_tol,
                                       start="dlarnv iseed=(1,3,5,7), info=1")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
