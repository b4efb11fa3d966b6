"""Diagnostics for the folded steps: dgks_worker runs under AHIP_FOLD / AHIP_FORCE_DGKS2."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for fx in sys.argv[1:]:
    for how, fold, force in [("rci", 1, 1), ("free", 0, 1), ("free", 1, 1), ("free", 0, 0), ("free", 1, 0), ("rci", 1, 0)]:
        out = f"/tmp/{fx}_{how}_{fold}_{force}.npz"
        env = dict(os.environ, AHIP_FOLD=str(fold), AHIP_FORCE_DGKS2=str(force))
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dgks_worker.py"), fx, how, out],
                           env=env, capture_output=True, text=True, timeout=120)
        if r.returncode:
            print(fx, how, fold, force, "FAILED", r.stderr[-1500:]); continue
        d = np.load(out)
        print(fx, how, "fold", fold, "force", force, {k: int(d[k]) for k in ("iters", "nopx", "nitref", "nrorth", "info")},
              "d[:3]", np.sort(d["d"])[-3:], flush=True)
