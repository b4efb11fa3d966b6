"""Run-to-run bitwise check of the row-distributed solve in deterministic mode
(ARPACK_HIP_DETERMINISTIC=1) per SpMV form, through tests/dist_worker.py at
P ranks on the host-staged transport: prints, per form, whether two runs give
bitwise equal Ritz values and Ritz-vector rows.

    python tools/det_dist_probe.py [P]
"""
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_dist import _run, _z  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
forms = [("full", "sym_csr", {}), ("sym_spill", "sym_csr_s", {"AHIP_DIST_SPILL": "1"}),
         ("sym_spill_free", "sym_csr_s", {})]
for det in ("1", "0"):
    for name, case, env in forms:
        env = dict(env, ARPACK_HIP_DETERMINISTIC=det)
        runs = []
        with tempfile.TemporaryDirectory() as td:
            for k in range(2):
                d = Path(td) / ("r%d" % k)
                d.mkdir()
                runs.append(_run(d, case, "g4_banded", P, extra_env=env))
        d0, d1 = runs[0][0]["d"], runs[1][0]["d"]
        z0, z1 = _z(runs[0]), _z(runs[1])
        print("det=%s %-15s P=%d d_bitwise=%s z_bitwise=%s max|dd|=%.2e" %
              (det, name, P, np.array_equal(d0, d1), np.array_equal(z0, z1),
               float(np.abs(d0 - d1).max())), flush=True)

# the product alone, repeated (dist_worker det_spmv)
for name, env in (("sym_spill", {"AHIP_DIST_SPILL": "1"}), ("sym_spill_free", {})):
    with tempfile.TemporaryDirectory() as td:
        ranks = _run(Path(td), "det_spmv", "-", P, extra_env=dict(env, ARPACK_HIP_DETERMINISTIC="1"))
    print("spmv %-15s sym=%s det=%s same=%s" % (name, [int(r["sym"][0]) for r in ranks],
                                                [int(r["det"][0]) for r in ranks],
                                                [bool(r["same"][0]) for r in ranks]), flush=True)
