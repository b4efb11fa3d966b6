"""Subprocess worker for tests/test_gpu_ztile_threads.py: products of config
5's operator family through the column-sorted tiles (n = 300,000, 40 entries a
row: the 4-slice packed form), default and deterministic mode, with the tile
workgroup size (AHIP_ZTILE_T) set by the caller.

    python tests/ztile_worker.py OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg  # noqa: E402


def main():
    out = sys.argv[1]
    pkg = load_pkg()
    n = 300_000
    Z = pkg.ZCSR.random(n, 40, 7, 40.0)
    rng = np.random.default_rng(4)
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 10.0 ** rng.uniform(-6, 0, n)
    y = Z.matvec(x)
    pkg.set_deterministic(True)
    yd = Z.matvec(x)
    pkg.set_deterministic(False)
    rp, col, val = Z.download()
    np.savez(out, y=y, yd=yd, x=x, rp=rp, col=col, val=val)


if __name__ == "__main__":
    main()
