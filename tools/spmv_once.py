"""Run one SpMV kernel variant a few times on the bench operator (for rocprofv3)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import load_pkg  # noqa: E402

pkg = load_pkg()
kernel = int(sys.argv[1]) if len(sys.argv) > 1 else 5
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
A = pkg.CSR.banded_sym(10_000_000, 1234, 4096, 25)
A.set_kernel(kernel, 4096)
print("ms", A.time_spmv(reps))
