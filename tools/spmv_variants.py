"""Time the SpMV kernel variants on the bench operator (hipEvents, back-to-back)."""
import json
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import load_pkg  # noqa: E402

pkg = load_pkg()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
A = pkg.CSR.banded_sym(n, 1234, 4096, 25)
by = 12.0 * A.nnz + 8.0 * (A.n + 1) + 16.0 * A.n
out = {}
for name, k, tile in [("vector", 0, 4096), ("stream2048", 1, 2048), ("stream4096", 1, 4096),
                      ("stream2048_nt", 2, 2048), ("stream4096_nt", 2, 4096),
                      ("window", 3, 4096), ("window_nt", 4, 4096), ("wvec", 5, 4096),
                      ("wvec_nt", 6, 4096), ("wvec8", 7, 4096), ("wvec_xcd", 8, 4096),
                      ("wvec_p3", 9, 4096), ("wvec_p4", 10, 4096),
                      ("wvec_again", 5, 4096), ("wvec_xcd_again", 8, 4096)]:
    if name.startswith("wvec"):
        pass
    A.set_kernel(k, tile)
    ms = min(A.time_spmv(10) for _ in range(3))
    out[name] = dict(ms=ms, gbs=by / (ms * 1e-3) / 1e9)
# correctness of every variant against the default kernel's output
import numpy as np  # noqa: E402
x = pkg.DeviceBuffer.from_numpy(np.random.default_rng(0).standard_normal(A.n))
y0, y1 = pkg.DeviceBuffer(A.n), pkg.DeviceBuffer(A.n)
A.set_kernel(8, 4096)
A.matvec_device(x.at(0), y0.at(0))
ref = y0.numpy()
for name, k in [("wvec", 5), ("wvec_p3", 9), ("wvec_p4", 10), ("window", 3)]:
    A.set_kernel(k, 4096)
    A.matvec_device(x.at(0), y1.at(0))
    out[name]["maxdiff"] = float(np.abs(y1.numpy() - ref).max())
print(json.dumps(out))
