"""SELL-64 vs the default LDS-window kernel on the bench operator: time (hipEvents,
back-to-back launches), effective GB/s over the algorithmic bytes, padding, and
max |y_sell - y_default|."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import load_pkg  # noqa: E402

pkg = load_pkg()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
A = pkg.CSR.banded_sym(n, 1234, 4096, 25)
alg = 10.0 * A.nnz + 8.0 * (A.n + 1) + 16.0 * A.n
x = pkg.DeviceBuffer.from_numpy(np.random.default_rng(0).standard_normal(A.n))
y0, y1 = pkg.DeviceBuffer(A.n), pkg.DeviceBuffer(A.n)
out = {"n": A.n, "nnz": A.nnz}
A.set_kernel(8, 4096)
A.matvec_device(x.at(0), y0.at(0))
ms = min(A.time_spmv(20) for _ in range(3))
out["wvec_xcd"] = dict(ms=ms, gbs=alg / (ms * 1e-3) / 1e9)
import ctypes as C  # noqa: E402
for u in (4, 5, 7, 3):
    t = time.time()
    A.set_kernel(11, u)
    if u == 4:
        out["sell_build_s"] = time.time() - t
        ns, pad = C.c_int64(), C.c_int64()
        L = pkg.lib()
        L.arpack_hip_csr_sell_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.arpack_hip_csr_sell_info(A.h, C.byref(ns), C.byref(pad))
        out["sell_slices"], out["sell_padding"] = ns.value, pad.value / A.nnz - 1.0
    A.matvec_device(x.at(0), y1.at(0))
    ms = min(A.time_spmv(20) for _ in range(3))
    r = dict(ms=ms, gbs=(10.0 * A.nnz + 20.0 * A.n) / (ms * 1e-3) / 1e9)
    d = np.abs(y1.numpy() - y0.numpy())
    r["maxdiff"] = float(d.max())
    out["sell_u%d" % u] = r
print(json.dumps(out))
