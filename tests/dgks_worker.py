"""Subprocess worker for tests/test_gpu_dgks.py: one dsaupd/dseupd solve on a
golden fixture (dnaupd/dneupd for a conv-diff fixture) through the free-running driver ("free": the second DGKS
refinement is resolved by the host, kFinDgks1Lazy) or the device-OP RCI loop
("rci": the gated in-stream refinement), with the environment (e.g.
AHIP_FORCE_DGKS2=1) set by the caller.

    python tests/dgks_worker.py FIXTURE {free|rci} OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import GOLDEN, load_pkg  # noqa: E402
from oracle import matrices as M  # noqa: E402


def main():
    fixture, how, out = sys.argv[1], sys.argv[2], sys.argv[3]
    g = dict(np.load(os.path.join(GOLDEN, fixture + ".npz"), allow_pickle=False))
    spec = g["spec"]
    pkg = load_pkg()
    if str(spec[0]) == "convdiff2d":  # dnaupd / dneupd (SRC/dnaitr.f's DGKS)
        A = pkg.CSR.convdiff2d(int(spec[1]), float(spec[2]))
        n = int(spec[1]) ** 2
        s = pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]),
                      mxiter=int(g["mxiter"]), v0=g["v0"], device=True)
        if how == "free":
            s.aupd_csr(A)
        else:
            while True:
                ido = s.aupd()
                if ido in (-1, 1):
                    A.matvec_device(s.slice(0), s.slice(1))
                elif ido == 99:
                    break
                else:
                    raise AssertionError(ido)
        nconv = int(s.iparam[4])
        dr, di, z, _ = s.eupd(rvec=True)
        st = pkg.stats()
        np.savez(out, d=dr[:nconv] + 1j * di[:nconv], z=z.numpy()[:nconv * n], ritz=s.ritz,
                 iters=int(s.iparam[2]), nopx=st["nopx"], nitref=st["nitref"],
                 nrorth=st["nrorth"], info=int(s.info[0]))
        return
    if str(spec[0]) == "banded_sym":
        rp, col, val = M.banded_sym(int(spec[1]), int(spec[2]), int(spec[3]), int(spec[4]))
    else:
        rp, col, val = M.anderson(int(spec[1]), int(spec[2]), float(spec[3]), int(spec[4]))
    A = pkg.CSR.from_arrays(rp, col, val)
    op = A if how == "free" else A.matvec_device
    d, z, res = pkg.eigsh(op, len(rp) - 1, int(g["nev"]), int(g["ncv"]), str(g["which"]),
                          float(g["tol"]), v0=g["v0"], mxiter=int(g["mxiter"]), device=True)
    st = pkg.stats()
    np.savez(out, d=d, z=z, iters=res["iters"], nopx=st["nopx"], nitref=st["nitref"],
             nrorth=st["nrorth"], info=res["info"])


if __name__ == "__main__":
    main()
