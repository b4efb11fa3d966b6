"""Restart-cycle throughput of the engine on BASELINE.json's other configs
(bench.py measures the north star; these are the parity configs at full size).

    python tools/bench_configs.py > profiles/r01_configs.json
    python tools/bench_configs.py C3      (only the configs whose name has C3)

C2  dsaupd, 2-D 5-pt Laplacian m = 1000 (n = 1e6), LA, nev 10, ncv 30
C3  dnaupd, 2-D convection-diffusion m = 1000 (rho = 10), LM, nev 10, ncv 40
C4  dsaupd, 3-D 7-pt Laplacian m = 215 (n = 9.94e6; the 1-GPU share of the
    8-GPU config is n/8 -- here the whole operator on one GPU), LA, nev 10, ncv 30
C5  znaupd, complex random CSR n = 5e5, 100 nnz/row, diag += 100, LM, in
    shift-invert mode 3 as BASELINE states it (OP = (A - sigma I)^{-1} by the
    device BiCGStab, tools/c5_mode3.py) and, for the Arnoldi engine alone, in
    mode 1 (OP = A)

Each real config: W warmup cycles, then K timed cycles (the engine parks at
cycle boundaries), device-synchronised; symmetric configs also with the
symmetric-storage SpMV.  C5: a capped solve (mxiter cycles) timed whole.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench import load_pkg  # noqa: E402

W, K = 2, 10


PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md), as bench.py


def roofline(prof):
    """Per-kernel-class GB/s of algorithmic bytes (kernel-mode hipEvents, as
    bench.py's roofline) and the SpMV's and SpMV + Gram-Schmidt's fraction of peak."""
    out = {k: dict(ms=v[0], launches=v[2], gbs=(v[1] / (v[0] * 1e-3) / 1e9) if v[0] > 0 else None)
           for k, v in prof.items() if v[2]}
    sp = prof.get("spmv", (0.0, 0.0, 0))
    # as bench.py: the finalize launches' time counts, their partial-sum bytes do not
    ms = sp[0] + sum(prof[k][0] for k in ("cgs_dots", "update", "place", "finalize"))
    by = sp[1] + sum(prof[k][1] for k in ("cgs_dots", "update", "place"))
    spmv_gbs = sp[1] / (sp[0] * 1e-3) / 1e9 if sp[0] > 0 else None
    step_gbs = by / (ms * 1e-3) / 1e9 if ms > 0 else None
    return dict(kernels=out, spmv_gbs=spmv_gbs, spmv_frac=spmv_gbs / PEAK_GBS if spmv_gbs else None,
                spmv_plus_orth_gbs=step_gbs,
                spmv_plus_orth_frac=step_gbs / PEAK_GBS if step_gbs else None, peak_gbs=PEAK_GBS)


def timed(pkg, s, A, ns=False):
    for k in (0, W):
        ido = s.aupd_cycles(A, k)
        if ido != 98:
            raise RuntimeError("solve ended early: ido %d info %d" % (ido, int(s.info[0])))
    pkg.synchronize()
    it0 = pkg.stats()["nopx"]
    t = time.perf_counter()
    ido = s.aupd_cycles(A, K)
    pkg.synchronize()
    el = time.perf_counter() - t
    nc = K if ido == 98 else int(s.iparam[2]) - W
    rec = dict(iters_per_s=nc / el, ms_per_cycle=1e3 * el / nc, cycles=nc,
               lanczos_steps_per_s=(pkg.stats()["nopx"] - it0) / el)
    if ido == 98:  # the next cycles with per-kernel events (out of the timed region)
        pkg.profile(True)
        pkg.profile_read()
        if s.aupd_cycles(A, min(K, 5)) in (98, 99):
            rec["roofline"] = roofline(pkg.profile_read())
        pkg.profile(False)
    return rec


def main():
    pkg = load_pkg()
    out = {}
    mx = W + K + 5
    only = sys.argv[1:]
    for name, make, which, ncv, ns in (
            ("C2_dsaupd_lap2d_1e6", lambda: pkg.CSR.laplace2d(1000), "LA", 30, False),
            ("C3_dnaupd_convdiff_1e6", lambda: pkg.CSR.convdiff2d(1000, 10.0), "LM", 40, True),
            ("C4_dsaupd_lap3d_9.94e6", lambda: pkg.CSR.laplace3d(215), "LA", 30, False)):
        if only and not any(o in name for o in only):
            continue
        A = make()
        n = A.n
        rec = dict(n=n, nnz=A.nnz, which=which, nev=10, ncv=ncv)
        cls = pkg.NsRci if ns else pkg.SymRci
        rec["full_storage"] = timed(pkg, cls(n, 10, ncv, which, 0.0, mxiter=mx, device=True), A, ns)
        if not ns:
            try:
                A.set_symmetric(True)
                rec["sym_storage"] = timed(pkg, cls(n, 10, ncv, which, 0.0, mxiter=mx, device=True), A)
            except RuntimeError as e:  # band wider than the LDS windows (3-D natural order)
                rec["sym_storage"] = "not applicable: %s" % e
        # the engine's form for this operator: the faster storage measured here
        forms = {k: rec[k] for k in ("full_storage", "sym_storage") if isinstance(rec.get(k), dict)}
        best = max(forms, key=lambda k: forms[k]["iters_per_s"])
        rec["best"] = dict(storage=best, iters_per_s=forms[best]["iters_per_s"],
                           spmv_plus_orth_frac=forms[best].get("roofline", {}).get("spmv_plus_orth_frac"))
        out[name] = rec
        print(json.dumps({name: rec}), file=sys.stderr, flush=True)
        del A
    if only and "C5" not in only:
        print(json.dumps(out), flush=True)
        return
    # C5 proxy: mode-1 znaupd on the config's operator, capped solve timed whole
    n = 500_000
    Z = pkg.ZCSR.random(n, 100, 5, 100.0)
    cap = 8
    s = pkg.ZRci(n, 10, 40, "LM", 0.0, mxiter=cap)
    pkg.synchronize()
    t = time.perf_counter()
    s.aupd_zcsr(Z)
    pkg.synchronize()
    el = time.perf_counter() - t
    out["C5_znaupd_zrandom_5e5_mode1"] = dict(
        n=n, per_row=100, which="LM", nev=10, ncv=40, cycles=int(s.iparam[2]), info=int(s.info[0]),
        seconds=el, iters_per_s_incl_setup=int(s.iparam[2]) / el,
        note="mode 1 (OP = A): the Arnoldi engine alone")
    del s, Z
    from c5_mode3 import run as run_mode3
    out["C5_znaupd_zrandom_5e5_mode3"] = run_mode3(pkg, cycles=4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
