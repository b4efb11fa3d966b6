"""Subprocess worker for tests/test_gpu_zfold.py: one free-running znaupd /
zneupd solve (mode 1, OP = the device complex CSR) on a complex golden fixture,
with the environment (AHIP_ZFOLD, AHIP_FORCE_DGKS2) set by the caller.

    python tests/zfold_worker.py FIXTURE OUT.npz
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import GOLDEN, load_pkg  # noqa: E402


def main():
    fixture, out = sys.argv[1], sys.argv[2]
    pkg = load_pkg()
    if fixture == "zdiag3":
        # a diagonal operator with 3 distinct eigenvalues: every Krylov space
        # closes after 3 steps (rnorm -> 0, the second refinement, then a
        # restart with a new start vector), inside folded cycles
        from oracle import matrices as M
        n = 3000
        lam = np.array([3 + 1j, 2.0 + 0j, 1 - 1j])[np.arange(n) % 3]
        Z = pkg.ZCSR.from_arrays(np.arange(n + 1), np.arange(n, dtype=np.int32), lam)
        g = dict(nev=2, ncv=8, which="LM", tol=1e-10, mxiter=300,
                 v0=M.dlarnv_uniform(2 * n)[0].view(np.complex128))
    else:
        g = dict(np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False))
        spec = g["spec"]
        Z = pkg.ZCSR.random(int(spec[1]), int(spec[2]), int(spec[3]), float(spec[4]))
    n = Z.n
    s = pkg.ZRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]),
                 mxiter=int(g["mxiter"]), v0=g["v0"])
    assert s.aupd_zcsr(Z) == 99
    d, z, nconv = s.eupd()
    st = pkg.stats()
    L = pkg.lib()
    L.arpack_hip_zfold_steps.restype = ctypes.c_longlong
    np.savez(out, d=d, z=z, ritz=s.ritz, iters=int(s.iparam[2]), nconv=nconv,
             nopx=int(s.iparam[8]), nrorth=int(s.iparam[10]), nitref=st["nitref"],
             nrstrt=st["nrstrt"],
             info=int(s.info[0]), folded=int(L.arpack_hip_zfold_steps()))


if __name__ == "__main__":
    main()
