"""Diagnostics for the folded Arnoldi steps (AHIP_FOLD_NS): dgks_worker runs."""
import os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for fx in sys.argv[1:]:
    res = {}
    for how, ns, force in [("rci", 1, 1), ("free", 1, 1), ("free", 0, 0), ("free", 1, 0)]:
        out = f"/tmp/{fx}_{how}_{ns}_{force}.npz"
        env = dict(os.environ, AHIP_FOLD_NS=str(ns), AHIP_FORCE_DGKS2=str(force))
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dgks_worker.py"), fx, how, out],
                           env=env, capture_output=True, text=True, timeout=200)
        if r.returncode:
            print(fx, how, ns, force, "FAILED", r.stderr[-1500:]); continue
        d = dict(np.load(out)); res[(how, ns, force)] = d
        print(fx, how, "ns", ns, "force", force, {k: int(d[k]) for k in ("iters", "nopx", "nitref", "nrorth", "info")}, flush=True)
    a, b = res.get(("rci", 1, 1)), res.get(("free", 1, 1))
    if a is not None and b is not None:
        print("  forced: d equal", np.array_equal(a["d"], b["d"]), "z equal", np.array_equal(a["z"], b["z"]))
    a, b = res.get(("free", 0, 0)), res.get(("free", 1, 0))
    if a is not None and b is not None:
        da, db = np.sort_complex(a["d"]), np.sort_complex(b["d"])
        print("  fold vs unfolded: max |d diff| / max|d|", np.abs(da - db).max() / np.abs(da).max())
