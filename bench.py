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
import signal
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


def visible_gpus() -> int:
    """GPUs this process may drive, counted without creating a HIP context in
    the launching process (torch.cuda.device_count() does not initialise the
    runtime on this image; it honours HIP_VISIBLE_DEVICES)."""
    import torch
    return int(torch.cuda.device_count())


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """`bench.py --gpus N` from a plain command (no WORLD_SIZE): start N rank
    processes, one per GPU, under torch.distributed.run -- the same form the
    driver uses for N > 1 -- before this process touches the GPU, wait for them,
    and forward rank 0's JSON line to stdout (everything else to stderr).
    Returns the exit status.  N above the visible GPU count is an error, unless
    --host-transport (a rehearsal: every rank on device 0)."""
    n = args.gpus
    if not args.host_transport:
        ndev = visible_gpus()
        if n > ndev:
            print(f"bench.py: --gpus {n} needs {n} GPUs, {ndev} visible (one rank per GPU; "
                  "--host-transport rehearses N ranks on one GPU)", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, text=True)

    def forward(signum, _frame):  # the launcher's own stop reaches every rank
        p.send_signal(signum)
    old = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    line = None
    try:
        for ln in p.stdout:
            s = ln.strip()
            if line is None and s.startswith("{"):
                try:
                    if "metric" in json.loads(s):
                        line = s
                        continue
                except ValueError:
                    pass
            sys.stderr.write(ln)
        rc = p.wait()
    finally:
        for sig, h in old.items():
            signal.signal(sig, h)
    if line is not None:
        print(line, flush=True)
    if rc == 0 and line is None:
        print("bench.py: the ranks ended without rank 0's JSON line", file=sys.stderr)
        rc = 1
    return rc


def kernel_family(name: str):
    """`k_csr_ssell` of 'void ahip::dev::(anonymous namespace)::k_csr_ssell<8, ...>(...)'."""
    import re
    m = re.search(r"(k_[A-Za-z0-9_]+)\s*[<(]", name)
    return m.group(1) if m else name


# the keys a PMC summary's workload block must share with the line it serves
PMC_KEYS = ("workload", "n", "nnz", "storage", "spmv_form")


def pmc_traffic(families, workload, profiles_dir=None):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3 PMC
    summary (profiles/r*_pmc.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected) OF THIS WORKLOAD: only a
    summary whose "workload" block equals `workload` on PMC_KEYS counts (the
    newest such file); the launch-weighted mean over the kernels whose family
    (template name) is in `families`.  Returns (bytes, file, None), or
    (None, None, reason)."""
    import glob
    d = profiles_dir or os.path.join(ROOT, "profiles")
    for f in sorted(glob.glob(os.path.join(d, "r*_pmc.json")), reverse=True):
        with open(f) as fh:
            doc = json.load(fh)
        w = doc.get("workload")
        if not isinstance(w, dict) or any(w.get(k) != workload.get(k) for k in PMC_KEYS):
            continue
        hits = [v for k, v in doc.get("kernels", {}).items() if kernel_family(k) in families]
        n = sum(v["launches"] for v in hits)
        if n:
            return sum(v["traffic_bytes"] * v["launches"] for v in hits) / n, os.path.basename(f), None
    return None, None, ("no committed PMC summary of this workload (%s) holds %s" %
                        (", ".join("%s=%s" % (k, workload.get(k)) for k in PMC_KEYS),
                         "/".join(sorted(families))))


def cpu_share():
    """Host cores for the CPU reference: the box's nproc, this process's affinity
    set, and the cgroup CPU quota (a GPU box's CPU share is a quota on a larger
    machine; more threads than the quota only oversubscribe it).  Threads used =
    min(affinity, quota); without a readable quota, min(affinity,
    OMP_NUM_THREADS) when the environment sets it."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(f) as fh:
                parts = fh.read().split()
            if f.endswith("cpu.max") and parts and parts[0] != "max":
                quota = int(parts[0]) / int(parts[1])
            elif f.endswith("quota_us") and parts and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                    quota = int(parts[0]) / int(fh.read().split()[0])
            if quota:
                break
        except (OSError, ValueError, IndexError):
            continue
    threads = aff
    if quota:
        threads = max(1, min(aff, int(quota)))
    elif os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = max(1, min(aff, int(os.environ["OMP_NUM_THREADS"])))
    return dict(nproc=os.cpu_count(), affinity=aff, cgroup_quota=quota, threads=threads)


def cpu_baseline(args, cycles):
    """The reference on the host cores (rank 0, N=1 only): restart cycles
    1..`cycles` of the same tol=eps solve the GPU's steady-state figure times,
    and (unless --no-cpu-ttc) the reference's full time-to-converge solve."""
    share = cpu_share()
    threads = share["threads"]
    cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--n", str(args.n), "--seed",
           str(args.seed), "--bandwidth", str(args.bandwidth), "--per-row", str(args.per_row),
           "--threads", str(threads), "--cycles", str(cycles)]
    if args.workload == "lap3d":
        cmd += ["--lap3d", str(args.m)]
    if not args.no_cpu_ttc:
        cmd.append("--ttc")
    try:
        # its own session, killed as a group afterwards: no descendant of the
        # baseline (BLAS / OpenMP helpers included) outlives bench.py
        p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             text=True, start_new_session=True)
        try:
            stdout, _ = p.communicate(timeout=900)
        finally:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()
        line = [ln for ln in stdout.splitlines() if ln.startswith("{")][-1]
        cb = json.loads(line)
        out = dict(value=cb["iters_per_s"], unit="iters/s", cores=threads, kind="reference",
                   sample=cb["sample"], lanczos_steps_per_s=cb["lanczos_steps_per_s"],
                   cycle_s=cb["cycle_s"], per_cycle_s=cb["per_cycle_s"], cycles=cb["cycles"],
                   host=share)
        if "time_to_converge" in cb:
            out["time_to_converge"] = cb["time_to_converge"]
        return out
    except Exception as e:  # report, never fake
        return dict(value=None, unit="iters/s", cores=threads, kind="reference", host=share,
                    sample="failed: %s" % (str(e)[:200]))


def ref_model_bytes(n, nnz, kev, kplusp):
    """SURVEY.md §8(d)'s byte model of the REFERENCE's arithmetic (full-CSR SpMV
    with int32 columns, four V passes per Lanczos step -- CGS + DGKS, taken on
    ~100% of steps here -- and dsapps' V*Q) for one restart cycle k = kev ->
    kplusp: returns (SpMV bytes per product, bytes per cycle)."""
    spmv = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n
    steps = sum(spmv + 32.0 * n * j + 48.0 * n for j in range(kev + 1, kplusp + 1))
    apps = 8.0 * n * (kplusp + kev + 1) + 16.0 * n
    return spmv, steps + apps


def comm_report(prof, D, dist, rank, ms_per_step):
    """The row-distributed engine's collectives in the profiled cycles: per rank
    and max over ranks, the device time per Lanczos step of the data-path RCCL
    allreduces (profiler class "allreduce": the Gram-Schmidt sums,
    PARPACK/SRC/MPI/pdsaitr.f:575-776) and of the SpMV's halo groups ("halo"),
    their counts per step, the kernels' time per step beside them, and
    comm_share = (allreduce + halo) per restart cycle / ms_per_step.  None on
    the single-GPU engine (no communicator)."""
    if D is None or not prof["spmv"][2]:
        return None
    steps = prof["spmv"][2]            # one SpMV (one halo group) per Lanczos step
    cyc = max(prof["vq"][2], 1)        # one V*Q per restart cycle
    ar_ms, _, ar_n = prof["allreduce"]
    h_ms, _, h_n = prof["halo"]
    kern_ms = sum(v[0] for k, v in prof.items() if k not in ("allreduce", "halo")) - h_ms
    mine = dict(rank=rank, lanczos_steps=steps, cycles=cyc,
                allreduce_us_per_step=1e3 * ar_ms / steps, allreduce_per_step=ar_n / steps,
                halo_us_per_step=1e3 * h_ms / steps, halo_per_step=h_n / steps,
                kernels_us_per_step=1e3 * kern_ms / steps,
                comm_ms_per_cycle=(ar_ms + h_ms) / cyc)
    ranks = [mine]
    if dist:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, mine)
    keys = ("allreduce_us_per_step", "halo_us_per_step", "kernels_us_per_step", "comm_ms_per_cycle")
    mx = {k: max(r[k] for r in ranks) for k in keys}
    return dict(per_rank=ranks, max_over_ranks=mx,
                comm_share=mx["comm_ms_per_cycle"] / ms_per_step if ms_per_step > 0 else None,
                measured_on="hipEvent marker spans on the engine's stream around each data-path "
                            "allreduce and each halo group, in the profiled cycles (not the timed "
                            "ones); the SpMV span holds its halo group, reported apart here",
                counts_note="allreduce_per_step and halo_per_step are launches per Lanczos step "
                            "(restart-cycle collectives included in the average)",
                baseline_note="a span's time includes its two marker packets (a 1-rank line's "
                              "halo group moves nothing and reads ~5 us a step: "
                              "profiles/r06a_force_dist.json) -- subtract that floor when "
                              "reading an N-rank line")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=("ns", "lap3d"), default="ns",
                    help="ns: the north-star banded symmetric CSR (n = --rows); lap3d: BASELINE "
                         "config 4, the 3-D 7-pt Laplacian m^3 (m = --lap-m), row-block / z-slab "
                         "sharded over the ranks (PARPACK/EXAMPLES/MPI/pdsdrv1.f)")
    ap.add_argument("--lap-m", dest="m", type=int, default=215,
                    help="lap3d grid edge (n = m^3; 215: 9.94e6); not --m, which torch.distributed.run "
                         "would take as an abbreviation of its own options")
    ap.add_argument("--rows", "--n", dest="n", type=int, default=10_000_000)
    ap.add_argument("--per-row", type=int, default=25)
    ap.add_argument("--bandwidth", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--nev", type=int, default=10)
    ap.add_argument("--ncv", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ttc", action="store_true")
    ap.add_argument("--no-cpu-ttc", action="store_true",
                    help="skip the reference's full time-to-converge solve on the host (~45 s)")
    ap.add_argument("--steady-cycles", type=int, default=3,
                    help="restart cycles 1..k of one solve timed on GPU and CPU alike")
    ap.add_argument("--no-full-storage", action="store_true",
                    help="skip the secondary full-storage and other-accumulator measurements of --storage sym")
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
    ap.add_argument("--sym-acc", choices=("fixed", "fp64"), default="fixed",
                    help="symmetric storage's transposed-term accumulator: fixed (the "
                         "fixed-point form, bitwise reproducible; default) or fp64 (LDS fp64 "
                         "atomics in schedule order); the other one runs beside as a companion")
    ap.add_argument("--deterministic", action="store_true",
                    help="deterministic mode (arpack_hip_set_deterministic): only fixed-order "
                         "SpMV forms (--storage sym: the fixed-point symmetric kernel "
                         "k_csr_ssell<..., DET = true>), so every solve is bitwise reproducible")
    args = ap.parse_args()
    if args.workload == "lap3d":
        args.n = args.m ** 3
        # the 7-pt Laplacian's top eigenvalues are clustered (multiplicities 3
        # and 6, gaps ~ 1/m^2): the tol = 1e-6 solve runs hundreds of cycles on
        # either side, so config 4's line is the restart-cycle rate only
        args.no_ttc = args.no_cpu_ttc = True
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # a plain `bench.py --gpus N`: become the launcher of N ranks (nothing
        # in this process has touched the GPU yet)
        sys.exit(launch_ranks(args, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(world_env or "1")
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher must start "
              "one rank per requested GPU", file=sys.stderr)
        sys.exit(2)
    dist = None
    out_fd = json_stdout()
    pkg = load_pkg()
    pkg.set_deterministic(args.deterministic)
    n, nev, ncv = args.n, args.nev, args.ncv
    D = None
    transport = "none"
    device = 0
    if world > 1:
        # control plane: gloo (CPU) hands rank 0's RCCL unique id to every rank;
        # the data path (allreduce of the Gram-Schmidt sums, SpMV halos) is RCCL.
        import torch.distributed as dist
        ndev = pkg.device_count()
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        if not args.host_transport and ndev < local_world:
            # every rank sees the same counts, so every rank leaves here
            print(f"bench.py rank {rank}: {local_world} ranks on this node but {ndev} GPUs "
                  "visible (one rank per GPU; --host-transport rehearses on one GPU)",
                  file=sys.stderr)
            sys.exit(2)
        dist.init_process_group("gloo")
        if args.host_transport:
            pkg.comm_init_host(world, rank, device=0)
            transport = "host-staged (gloo)"
        else:
            box = [pkg.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            # one GPU per rank; a launcher that narrows each rank's visible
            # devices (HIP_VISIBLE_DEVICES) leaves device 0 = this rank's GPU
            device = local_rank % max(1, ndev)
            pkg.comm_init(world, rank, box[0], device=device)
            transport = "rccl"
        r0, r1 = pkg.partition_rows(n, world, rank)
    else:
        r0, r1 = 0, n
        if args.force_dist:
            pkg.comm_init(1, 0, pkg.comm_unique_id(), device=0)
            transport = "rccl"
    # which GPU every rank drove, and how many ranks the engine's communicator has
    comm_ranks = pkg.comm_size() if transport != "none" else 1
    devices = [dict(rank=rank, device=device, pci_bus_id=pkg.pci_bus_id(device),
                    comm_ranks=comm_ranks)]
    if dist:
        allr = [None] * world
        dist.all_gather_object(allr, devices[0])
        devices = allr
    t = time.time()
    if args.workload == "lap3d":  # this rank's z-slab rows, global columns
        A = pkg.CSR.laplace3d(args.m, 1.0, r0, r1)
    else:
        A = pkg.CSR.banded_sym(n, args.seed, args.bandwidth, args.per_row, r0, r1)
    if world > 1 or args.force_dist:
        D = pkg.DistOp(A, n, r0)
    storage = "full"
    if args.storage == "sym":  # row blocks: upper-triangle SpMV + forward spill exchange
        try:
            # collective on a distributed operator: every rank ends up in the
            # same mode (all fall back to full storage if any rank's plan fails)
            A.set_symmetric(True)
            storage = "sym" if A.symmetric else "full"
        except RuntimeError:
            pass
    # the symmetric kernel's accumulator: the fixed-point form by default (y
    # bitwise reproducible), --sym-acc fp64 the LDS fp64 atomics
    if storage == "sym":
        A.set_sym_accumulator(args.sym_acc)
    sym_form = A.sym_form
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
    acc_companion = None
    if storage == "sym" and world == 1 and not args.no_full_storage and not args.deterministic:
        # the same K cycles with the OTHER accumulator of the symmetric kernel
        # (fixed point <-> LDS fp64 atomics), reported beside
        other = "fp64" if args.sym_acc == "fixed" else "fixed"
        A.set_sym_accumulator(other)
        if A.sym_form != sym_form:
            s_d, ido_d, el_d, nopx_d, _ = timed_run()
            acc_companion = dict(accumulator=other, value=args.steps / el_d,
                                 ms_per_step=1e3 * el_d / args.steps,
                                 lanczos_steps_per_s=nopx_d / el_d,
                                 bitwise_reproducible=A.sym_form == "sym_fixed")
            del s_d
        else:
            acc_companion = dict(accumulator=other, value=None,
                                 note="operator outside the fixed-point form")
        A.set_sym_accumulator(args.sym_acc)
    s, ido, elapsed, nopx, nsolves = timed_run()
    # Per-kernel roofline: the next K cycles of the same solve with hipEvents on
    # every kernel's dispatch (start event on a span's first kernel, stop event
    # on its last: hipExtLaunchKernel), kept out of the timed region above; if that solve has
    # finished, min(K, 10) cycles of a fresh one after its warmup.
    prof = None
    prof_cycles = None
    if not args.no_profile:
        pk = args.steps
        prof_cycles = "the %d cycles after the timed ones, same solve" % pk
        if ido != 98:
            del s
            s, _ = warm_solve(min(args.warmup, 5))
            pk = min(args.steps, 10)
            prof_cycles = ("%d cycles of a fresh solve after %d warmup cycles (the timed solve "
                           "had converged)" % (pk, min(args.warmup, 5)))
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
    steady = None
    v0 = None
    if not args.no_ttc or args.steady_cycles > 0:
        iseed = np.array([1, 3, 5, 7], np.int32)
        v0 = np.empty(n, np.float64)
        pkg.lib().arpack_hip_kit_dlarnv(iseed.ctypes.data_as(pkg.C.POINTER(pkg.C.c_int)), n,
                                        v0.ctypes.data_as(pkg.C.POINTER(pkg.C.c_double)))
    # ---- steady state over IDENTICAL cycles: restart cycles 1..k of the tol = eps
    # solve from the reference's first draw -- the very cycles the CPU baseline
    # times -- each parked and drained; np of each cycle from the OP*x counts
    if args.steady_cycles > 0:
        s3 = pkg.SymRci(nloc, nev, ncv, "LA", 0.0, mxiter=300, device=True, v0=v0[r0:r1])
        assert cycles(s3, 0) == 98
        pkg.synchronize()
        if dist:
            dist.barrier()
        nops = []
        t = time.perf_counter()
        for _ in range(args.steady_cycles):
            o0 = pkg.stats()["nopx"]
            if cycles(s3, 1) != 98:
                break
            nops.append(pkg.stats()["nopx"] - o0)
        pkg.synchronize()
        secs = time.perf_counter() - t
        if dist:
            tt = torch.tensor([secs], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            secs = float(tt.item())
        if len(nops) == args.steady_cycles:
            steady = dict(cycles="1..%d" % len(nops), seconds=secs, iters_per_s=len(nops) / secs,
                          ms_per_cycle=1e3 * secs / len(nops), lanczos_steps=nops,
                          lanczos_steps_per_s=sum(nops) / secs,
                          start="dlarnv iseed=(1,3,5,7), tol = eps")
        del s3
    if not args.no_ttc:
        s2 = pkg.SymRci(nloc, nev, ncv, "LA", 1e-6, mxiter=300, device=True, v0=v0[r0:r1])
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
    del v0

    if prof is None:
        prof = {k: (0.0, 0.0, 0) for k in pkg.PROF_CLASSES}
    ms, by, cnt = prof["spmv"]
    if D is not None:
        # a row-distributed SpMV is a marker span holding its halo group: the
        # kernel's own time is the span less the halo's
        ms = max(ms - prof["halo"][0], 0.0)
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

    # counter traffic from a committed PMC summary of THIS workload (same
    # operator, size, storage and mode), single GPU only
    # (one symmetric kernel, k_csr_ssell<..., DET, ...>, since round 6; the
    # fixed-point form's former name is kept for older summaries -- the
    # workload's "spmv_form" key tells the two accumulators apart)
    families = {"k_csr_ssell", "k_csr_ssell_det"} if storage == "sym" \
        else {"k_csr_sell", "k_csr_sell_fin"}
    wl = dict(workload=args.workload, n=n, nnz=nnz, storage=storage, spmv_form=sym_form)
    if world == 1 and D is None:
        traffic, traffic_src, traffic_note = pmc_traffic(families, wl)
    else:
        traffic, traffic_src, traffic_note = None, None, "PMC summaries are single-GPU runs"
    comm_prof = comm_report(prof, D, dist, rank, 1e3 * elapsed / args.steps)
    if args.workload == "lap3d":
        wl_name = ("dsaupd LA on the 3-D 7-pt Laplacian m=%d, n=%d (BASELINE config 4, "
                   "pdsaupd-equivalent row-block / z-slab sharding)" % (args.m, n))
        data = "synthetic (3-D 7-pt Laplacian generated in HBM, each rank its own z-slab rows)"
    else:
        wl_name = "dsaupd LA on NS symmetric CSR (BASELINE north star)"
        data = "synthetic (NS operator generated in HBM from a counter hash; no files)"
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
        "data": data,
        "config": {"workload": wl_name, "workload_key": args.workload,
                   "n": n, "nnz": nnz, "nnz_per_row": nnz / n, "nev": nev, "ncv": ncv,
                   "which": "LA", "tol": "eps (a solve that converges inside the timed window is followed by a fresh one)",
                   "spmv_storage": "symmetric (upper triangle)" if storage == "sym" else "full CSR",
                   # full storage and the symmetric kernel's fixed-point form: fixed-
                   # order sums throughout; the fp64 accumulator's transposed terms
                   # meet in LDS in wave order (Ritz values to ~6e-15, not bitwise)
                   "spmv_form": sym_form,
                   "bitwise_reproducible": sym_form in ("full", "sym_fixed"),
                   "deterministic_mode": bool(args.deterministic),
                   "parallelism": "single GPU" if world == 1 else
                   f"row-block x{world} (RCCL allreduce + halo)" if not args.host_transport else
                   f"REHEARSAL row-block x{world} on one GPU, host-staged gloo transport"},
        "comm": {"transport": transport, "ranks": comm_ranks,
                 "distinct_gpus": len({d["pci_bus_id"] for d in devices}), "ranks_devices": devices},
        "rccl_ranks": comm_ranks if transport == "rccl" else 0,
        "lanczos_steps_per_s": nopx / elapsed,
        "solves_in_timed_region": nsolves,
        "time_to_converge": ttc,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                     "traffic_source": traffic_src, "traffic_note": traffic_note,
                     "traffic_ratio": (traffic / spmv_bytes) if traffic and spmv_bytes else None,
                     "kernel": ("csr_spmv symmetric storage (k_csr_ssell: upper-triangle SELL-64 "
                                "slices over LDS x/y windows, 16-bit window-relative cols, the "
                                "transposed terms " + ("as 64-bit fixed-point LDS sums (bitwise "
                                                       "reproducible)" if sym_form == "sym_fixed"
                                                       else "as LDS fp64 atomics") +
                                "; on one GPU the chain-head combine and the step's deferred "
                                "finalize run inside it, else k_ssell_combine follows)")
                               if storage == "sym"
                               else ("csr_spmv (k_csr_sell: SELL-64 length-sorted slices over LDS "
                                     "x windows, 16-bit window-relative cols, XCD-contiguous "
                                     "superblocks)"),
                     "measured_on": "hipEvents attached to the SpMV kernels' own dispatches "
                                    "(hipExtLaunchKernel start/stop: kernel execution time, as "
                                    "rocprofv3's kernel trace measures it) over a second run of the "
                                    "same K cycles (events kept out of the timed region)",
                     "read_stream_measured": READ_STREAM_GBS,
                     "frac_of_read_stream": (achieved / READ_STREAM_GBS) if achieved else None,
                     "bytes_model": ("engine bytes: what the dominant kernel must move in "
                                     "ITS storage -- upper triangle only, 10 B per stored entry "
                                     "(8 B value + 2 B window-relative column), x and y 8n each, "
                                     "+ 4n (the row map) + combine slots; not the reference's "
                                     "12 B per entry of the full CSR (see reference_model)"
                                     if storage == "sym" else
                                     "engine bytes: full CSR in SELL-64 slices, 10 B per stored "
                                     "entry (8 B value + 2 B window-relative column), x and y 8n "
                                     "each, + 4n row map"),
                     "reference_model": None,
                     "bytes_per_launch": spmv_bytes, "avg_launch_ms": spmv_avg_ms,
                     # the per-kernel profile is not the timed cycles themselves:
                     # later cycles run more Lanczos steps per cycle as nev grows
                     "profiled_cycles": prof_cycles,
                     # (one V*Q a restart: a solve that converges inside the
                     # profiled window runs fewer than requested)
                     "profiled_steps_per_cycle": (cnt / prof["vq"][2]) if cnt and prof["vq"][2] else None,
                     "timed_steps_per_cycle": nopx / args.steps,
                     "spmv_plus_orth_gbs": step_gbs,
                     "spmv_plus_orth_frac": (step_gbs / HBM_PEAK_GBS) if step_gbs else None},
        "kernels": kernels,
        "comm_profile": comm_prof,
        "gen_s": gen_s,
        "storage": storage,
        "full_storage": full_storage,
        "accumulator_companion": acc_companion,
    }
    # SURVEY.md §8(d)'s byte model of the reference's arithmetic on the same
    # product / cycle, divided by OUR times: an "effective" rate that can exceed
    # the HBM peak, because the engine moves fewer bytes (upper-triangle storage,
    # 16-bit columns, two V passes a step instead of four)
    rs, rc = ref_model_bytes(n, nnz, nev, ncv)
    out["roofline"]["reference_model"] = {
        "spmv_bytes": rs, "cycle_bytes": rc,
        "spmv_effective_gbs": rs / (spmv_avg_ms * 1e-3) / 1e9 if cnt else None,
        "cycle_effective_gbs": (rc / (steady["ms_per_cycle"] * 1e-3) / 1e9) if steady else None,
        "cycle": "k = %d -> %d (the steady cycles 1..k, np = %d)" % (nev, ncv, ncv - nev),
        "definition": "SpMV 12 nnz + 4(n+1) + 16n; per Lanczos step j: + 32 n j (CGS + DGKS "
                      "over V(:,1:j)) + 48 n; per cycle + 8n(kplusp + kev + 1) + 16n (V*Q)"}
    if steady:
        out["steady_state"] = steady
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        del A
        out["cpu_baseline"] = cpu_baseline(args, args.steady_cycles if steady else 1)
        cb = out["cpu_baseline"]
        if steady and cb.get("value"):
            steady["cpu_iters_per_s"] = cb["value"]
            steady["speedup_same_cycles"] = steady["iters_per_s"] / cb["value"]
        if ttc and cb.get("time_to_converge"):
            ttc["cpu_seconds"] = cb["time_to_converge"]["seconds"]
            ttc["speedup"] = cb["time_to_converge"]["seconds"] / ttc["seconds"]
            ttc["cpu_same_solve"] = (cb["time_to_converge"]["iters"] == ttc["iters"] and
                                     cb["time_to_converge"]["nopx"] == ttc["nopx"])
        if out["cpu_baseline"].get("value"):
            out["speedup_vs_cpu"] = iters_per_s / out["cpu_baseline"]["value"]
            # per Lanczos step (OP*x): the GPU's timed cycles run the adapted np
            # of the solve (nev grows), the CPU sample cycles 1..k of np = 20
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
