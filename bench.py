#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json `metric`): implicit-restart (Arnoldi)
iterations per second of the MI355X engine's dsaupd on the north-star operator

    NS: symmetric CSR, n = 10,000,000 rows, ~50 nnz/row (banded hash pattern,
        bandwidth 4096), diagonally dominant Anderson-like, which='LA',
        nev = 10, ncv = 30, fp64, generated directly in HBM (synthetic data).

A "step" is ONE implicit-restart cycle = one increment of iparam(3): np = 20
Lanczos steps (CSR SpMV + classical Gram-Schmidt + DGKS against V, the DGKS
sweep folded into the next step's passes: two passes over V per step, DESIGN.md
§2) followed by the host shift selection and the on-device V*Q update (dsapps).
The whole loop runs on the GPU through arpack_hip_dsaupd_csr_cycles (the engine
parks every K cycles so exactly K cycles sit inside the timed region).

OP: the operator is symmetric (dsaupd's contract), so by default the CSR is
declared symmetric and the SpMV streams only its upper triangle
(arpack_hip_csr_set_symmetric); the full-storage SpMV (bitwise SciPy's
csr_matvec) runs the same K cycles beside it and is reported as `full_storage`.

Also reported: Lanczos steps/s (OP*x/s), time-to-converge at tol=1e-6, the
roofline of the dominant kernel (SpMV) from live hipEvent timing, and the
reference CPU path (oracle/_ref: arpack-ng Fortran + OpenBLAS, OpenMP SpMV)
timed on a bounded sample on the host cores.

    python bench.py [--gpus N] [--steps K] [--warmup W]
Multi-GPU: launched by torch.distributed.run, one rank per GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# measured read-stream ceiling in the Gram-Schmidt pass shape (tools/stream_bench.hip,
# profiles/r02_stream_bench.txt: 20 columns x 1e7 rows, 8-B non-temporal loads,
# 6.6-6.9 TB/s across boxes); the guide's copy figure is 6.29 TB/s
READ_STREAM_GBS = 6700.0


def load_pkg():
    import importlib.util
    if "arpack_ng_amd" in sys.modules:
        return sys.modules["arpack_ng_amd"]
    d = os.path.join(ROOT, "arpack-ng_amd")
    spec = importlib.util.spec_from_file_location("arpack_ng_amd", os.path.join(d, "__init__.py"),
                                                  submodule_search_locations=[d])
    m = importlib.util.module_from_spec(spec)
    sys.modules["arpack_ng_amd"] = m
    spec.loader.exec_module(m)
    return m


def json_stdout():
    """stdout carries exactly ONE JSON line (rank 0's; the driver's contract).
    Everything else that writes to fd 1 -- RCCL's version banner at
    communicator init, gloo's "[Gloo] Rank r is connected ..." from every rank,
    library prints -- is sent to stderr: fd 1 is pointed at stderr for the
    whole run and the JSON goes to a saved duplicate of the original stdout."""
    import ctypes
    sys.stdout.flush()
    ctypes.CDLL(None).fflush(None)
    fd = os.dup(1)
    os.dup2(2, 1)
    return fd


def pmc_traffic(kernel_substr: str):
    """HBM bytes per launch of `kernel_substr` from the committed rocprofv3 PMC
    summary (profiles/r*_pmc.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes of this same command, gfx950-corrected)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as fh:
        ks = json.load(fh)["kernels"]
    hits = [v for k, v in ks.items() if kernel_substr in k]
    if not hits:
        return None, None
    v = max(hits, key=lambda e: e["launches"])
    return v["traffic_bytes"], os.path.basename(files[-1])


def cpu_baseline(args):
    """The reference on the host cores (rank 0, N=1 only), bounded sample."""
    threads = min(16, len(os.sched_getaffinity(0)))
    cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--n", str(args.n), "--seed",
           str(args.seed), "--bandwidth", str(args.bandwidth), "--per-row", str(args.per_row),
           "--threads", str(threads)]
    try:
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        cb = json.loads(line)
        return dict(value=cb["iters_per_s"], unit="iters/s", cores=threads, kind="reference",
                    sample=cb["sample"], lanczos_steps_per_s=cb["lanczos_steps_per_s"],
                    cycle_s=cb["cycle_s"])
    except Exception as e:  # report, never fake
        return dict(value=None, unit="iters/s", cores=threads, kind="reference",
                    sample="failed: %s" % (str(e)[:200]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", "--n", dest="n", type=int, default=10_000_000)
    ap.add_argument("--per-row", type=int, default=25)
    ap.add_argument("--bandwidth", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--nev", type=int, default=10)
    ap.add_argument("--ncv", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ttc", action="store_true")
    ap.add_argument("--no-full-storage", action="store_true",
                    help="skip the secondary full-storage measurement of --storage sym")
    ap.add_argument("--host-transport", action="store_true",
                    help="rehearsal only: engine collectives over gloo instead of RCCL, so N ranks "
                         "can share one GPU (every rank uses device 0)")
    ap.add_argument("--storage", choices=("sym", "full"), default="sym",
                    help="sym: the operator is declared symmetric (dsaupd's contract) and the "
                         "SpMV streams its upper triangle (arpack_hip_csr_set_symmetric); full: "
                         "full CSR, bitwise SciPy's csr_matvec.")
    ap.add_argument("--force-dist", action="store_true",
                    help="measurement aid: with one rank, still run the row-distributed engine "
                         "(1-rank RCCL communicator, DistOp) to price its machinery")
    ap.add_argument("--no-profile", action="store_true",
                    help="no per-kernel hipEvents in the timed region (overhead check)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    out_fd = json_stdout()
    pkg = load_pkg()
    n, nev, ncv = args.n, args.nev, args.ncv
    D = None
    if world > 1:
        # control plane: gloo (CPU) hands rank 0's RCCL unique id to every rank;
        # the data path (allreduce of the Gram-Schmidt sums, SpMV halos) is RCCL.
        import torch.distributed as dist
        dist.init_process_group("gloo")
        if args.host_transport:
            pkg.comm_init_host(world, rank, device=0)
        else:
            box = [pkg.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            # one GPU per rank; a launcher that narrows each rank's visible
            # devices (HIP_VISIBLE_DEVICES) leaves device 0 = this rank's GPU
            pkg.comm_init(world, rank, box[0], device=local_rank % max(1, pkg.device_count()))
        r0, r1 = pkg.partition_rows(n, world, rank)
    else:
        r0, r1 = 0, n
        if args.force_dist:
            pkg.comm_init(1, 0, pkg.comm_unique_id(), device=0)
    t = time.time()
    A = pkg.CSR.banded_sym(n, args.seed, args.bandwidth, args.per_row, r0, r1)
    if world > 1 or args.force_dist:
        D = pkg.DistOp(A, n, r0)
    storage = "full"
    if args.storage == "sym":  # row blocks: upper-triangle SpMV + forward spill exchange
        try:
            # collective on a distributed operator: every rank ends up in the
            # same mode (all fall back to full storage if any rank's plan fails)
            A.set_symmetric(True)
            storage = "sym"
        except RuntimeError:
            pass
    gen_s = time.time() - t
    nnz = A.nnz
    if dist:
        import torch
        tn = torch.tensor([nnz], dtype=torch.int64)
        dist.all_reduce(tn)
        nnz = int(tn.item())
    nloc = r1 - r0

    def solver(tol, mxiter):
        return pkg.SymRci(nloc, nev, ncv, "LA", tol, mxiter=mxiter, device=True)

    def cycles(s, k):
        return pkg.pdsaupd_cycles(s, D, k) if D is not None else s.aupd_cycles(A, k)

    # ---- restart-cycle throughput: W untimed cycles, then exactly K timed ones.
    # At tol = eps the NS solve converges after ~25 cycles; if it does so inside
    # the timed region, the remaining cycles run on a fresh solve (pre-allocated;
    # its start vector and initial factorisation are timed too), so K is always
    # exactly K restart cycles.
    def warm_solve(w):
        """A solve after w untimed restart cycles, and the cycles it has done
        (a solve that converges inside the warmup is replaced by a fresh one)."""
        s = solver(0.0, 300)
        assert cycles(s, 0) == 98                # getv0 + initial nev-step factorization
        done = 0
        while w > 0:
            if cycles(s, w) == 98:
                done += w
                break
            w -= int(s.iparam[2]) - done         # converged after that many more cycles
            s = solver(0.0, 300)
            assert cycles(s, 0) == 98
            done = 0
        return s, done

    def timed_run():
        s, wdone = warm_solve(args.warmup)       # warmup cycles
        spare = solver(0.0, 300)
        pkg.synchronize()
        if dist:
            dist.barrier()
        it0 = pkg.stats()["nopx"]
        t0 = time.perf_counter()
        ido = cycles(s, args.steps)              # the timed region: nothing but the solve
        cur, nopx, nsolves = s, 0, 1
        left = 0 if ido == 98 else args.steps - (int(s.iparam[2]) - wdone)
        while True:
            nopx += pkg.stats()["nopx"] - it0    # dstats restarts with every solve
            if left <= 0:
                break
            cur, spare = (spare if spare is not None else solver(0.0, 300)), None
            nsolves += 1
            cycles(cur, 0)
            it0 = 0
            ido = cycles(cur, left)
            left = 0 if ido == 98 else left - int(cur.iparam[2])
        pkg.synchronize()
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        del spare
        return cur, ido, t1 - t0, nopx, nsolves

    full_storage = None
    if storage == "sym" and world == 1 and not args.no_full_storage:
        # the same K cycles with the full-storage (bitwise csr_matvec) SpMV, reported beside
        A.set_symmetric(False)
        s_f, ido_f, el_f, nopx_f, _ = timed_run()
        full_storage = dict(value=args.steps / el_f, ms_per_step=1e3 * el_f / args.steps,
                            lanczos_steps_per_s=nopx_f / el_f)
        del s_f
        A.set_symmetric(True)
    s, ido, elapsed, nopx, nsolves = timed_run()
    # Per-kernel roofline: the next K cycles of the same solve with hipEvents on
    # every kernel's dispatch (start event on a span's first kernel, stop event
    # on its last: hipExtLaunchKernel), kept out of the timed region above; if that solve has
    # finished, min(K, 10) cycles of a fresh one after its warmup.
    prof = None
    if not args.no_profile:
        pk = args.steps
        if ido != 98:
            del s
            s, _ = warm_solve(min(args.warmup, 5))
            pk = min(args.steps, 10)
        pkg.profile(True)
        pkg.profile_read()
        cycles(s, pk)
        prof = pkg.profile_read()
        pkg.profile(False)
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ncycles = args.steps
    iters_per_s = ncycles / elapsed
    del s

    # ---- time to converge (tol = 1e-6), full solve incl. start vector.  The
    # start vector is the reference's first draw in a fresh process (dlarnv,
    # iseed = 1,3,5,7: SRC/dgetv0.f:202-208) whatever this process drew before,
    # so the solve is the same for every --steps / --warmup / --gpus: the
    # full-size GPU test checks this case against the reference (11 cycles,
    # 187 OP*x).  Generated on the host (80 MB) and sliced per rank.
    ttc = None
    if not args.no_ttc:
        iseed = np.array([1, 3, 5, 7], np.int32)
        v0 = np.empty(n, np.float64)
        pkg.lib().arpack_hip_kit_dlarnv(iseed.ctypes.data_as(pkg.C.POINTER(pkg.C.c_int)), n,
                                        v0.ctypes.data_as(pkg.C.POINTER(pkg.C.c_double)))
        s2 = pkg.SymRci(nloc, nev, ncv, "LA", 1e-6, mxiter=300, device=True, v0=v0[r0:r1])
        del v0
        pkg.synchronize()
        if dist:
            dist.barrier()
        t = time.perf_counter()
        cycles(s2, -1)
        pkg.synchronize()
        secs = time.perf_counter() - t
        if dist:
            tt = torch.tensor([secs], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            secs = float(tt.item())
        ttc = dict(seconds=secs, iters=int(s2.iparam[2]), nconv=int(s2.iparam[4]),
                   nopx=int(s2.iparam[8]), info=int(s2.info[0]), tol=1e-6,
                   start="dlarnv iseed=(1,3,5,7): the reference's first solve in a fresh process")
        del s2

    if prof is None:
        prof = {k: (0.0, 0.0, 0) for k in ("spmv", "cgs_dots", "update", "vq", "place",
                                           "finalize", "other")}
    ms, by, cnt = prof["spmv"]
    spmv_avg_ms = ms / max(cnt, 1)
    spmv_bytes = by / max(cnt, 1)
    achieved = spmv_bytes / (spmv_avg_ms * 1e-3) / 1e9 if cnt else None
    kernels = {k: dict(ms=v[0], launches=v[2],
                       gbs=(v[1] / (v[0] * 1e-3) / 1e9) if v[0] > 0 and v[1] > 0 else None)
               for k, v in prof.items()}
    orth_ms = sum(prof[k][0] for k in ("cgs_dots", "update", "finalize", "place"))
    orth_bytes = sum(prof[k][1] for k in ("cgs_dots", "update", "place"))
    step_ms = ms + orth_ms
    step_gbs = (by + orth_bytes) / (step_ms * 1e-3) / 1e9 if step_ms > 0 else None

    # PMC traffic is collected on the default single-GPU workload only
    spmv_kernel = "k_csr_ssell" if storage == "sym" else "k_csr_sell"
    traffic, traffic_src = (pmc_traffic(spmv_kernel) if world == 1 and n == 10_000_000
                            else (None, None))
    out = {
        "metric": "Arnoldi iters/sec + time-to-converge (nev=10), n=10M CSR; %HBM roofline",
        "value": iters_per_s,
        "unit": "iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / ncycles,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (NS operator generated in HBM from a counter hash; no files)",
        "config": {"workload": "dsaupd LA on NS symmetric CSR (BASELINE north star)",
                   "n": n, "nnz": nnz, "nnz_per_row": nnz / n, "nev": nev, "ncv": ncv,
                   "which": "LA", "tol": "eps (a solve that converges inside the timed window is followed by a fresh one)",
                   "spmv_storage": "symmetric (upper triangle)" if storage == "sym" else "full CSR",
                   "parallelism": "single GPU" if world == 1 else
                   f"row-block x{world} (RCCL allreduce + halo)" if not args.host_transport else
                   f"REHEARSAL row-block x{world} on one GPU, host-staged gloo transport"},
        "lanczos_steps_per_s": nopx / elapsed,
        "solves_in_timed_region": nsolves,
        "time_to_converge": ttc,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "kernel": ("csr_spmv symmetric storage (k_csr_ssell + k_ssell_combine: "
                                "upper-triangle SELL-64 slices over LDS x/y windows, LDS atomic "
                                "transposed terms, 16-bit window-relative cols)") if storage == "sym"
                               else ("csr_spmv (k_csr_sell: SELL-64 length-sorted slices over LDS "
                                     "x windows, 16-bit window-relative cols, XCD-contiguous "
                                     "superblocks)"),
                     "measured_on": "hipEvents attached to the SpMV kernels' own dispatches "
                                    "(hipExtLaunchKernel start/stop: kernel execution time, as "
                                    "rocprofv3's kernel trace measures it) over a second run of the "
                                    "same K cycles (events kept out of the timed region)",
                     "read_stream_measured": READ_STREAM_GBS,
                     "frac_of_read_stream": (achieved / READ_STREAM_GBS) if achieved else None,
                     "bytes_per_launch": spmv_bytes, "avg_launch_ms": spmv_avg_ms,
                     "spmv_plus_orth_gbs": step_gbs,
                     "spmv_plus_orth_frac": (step_gbs / HBM_PEAK_GBS) if step_gbs else None},
        "kernels": kernels,
        "gen_s": gen_s,
        "storage": storage,
        "full_storage": full_storage,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del A
        out["cpu_baseline"] = cpu_baseline(args)
        if out["cpu_baseline"].get("value"):
            out["speedup_vs_cpu"] = iters_per_s / out["cpu_baseline"]["value"]
            # per Lanczos step (OP*x): the GPU's timed cycles run the adapted np
            # of the solve (nev grows), the CPU sample a first cycle of np = 20
            out["speedup_vs_cpu_lanczos_steps"] = \
                (nopx / elapsed) / out["cpu_baseline"]["lanczos_steps_per_s"]
    if rank == 0:
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    if dist or args.force_dist:
        del D
        pkg.comm_destroy()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
