"""Achievable HBM read bandwidth on this device (8- vs 16-byte loads per lane)."""
import ctypes as C
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import load_pkg  # noqa: E402

L = load_pkg().lib()
L.arpack_hip_stream_probe.restype = C.c_double
L.arpack_hip_stream_probe.argtypes = [C.c_int64, C.c_int, C.c_int, C.c_int]
out = {}
for w in (8, 16):
    for g in (1024, 2048, 4096, 8192, 16384):
        out[f"w{w}_g{g}"] = L.arpack_hip_stream_probe(4 << 30, w, g, 10)
print(json.dumps(out))
