"""Probe: dnaupd's complex-shift fixtures (m10, m11) through the engine --
host RCI with the reference's caller (complex LU on the host) and the device
pair (direct tridiagonal solve, BiCGStab) -- printing restart cycles and OP*x."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bench import load_pkg  # noqa: E402
import modes  # noqa: E402


def dev(pkg, S):
    S = S.tocsr()
    S.sort_indices()
    return pkg.CSR.from_arrays(S.indptr, S.indices, S.data)


def main():
    pkg = load_pkg()
    for name in ("m10_ns_cshift_re", "m11_ns_cshift_im"):
        g = dict(np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False))
        mode, n = int(g["mode"]), int(g["n"])
        sigma = complex(float(g["sigmar"]), float(g["sigmai"]))
        c = modes.CShiftCaller(mode, n, sigma)
        s = pkg.NsRci(n, 4, 20, "LM", 1e-10, bmat="G", mode=mode, mxiter=300, v0=g["v0"])
        while True:
            ido = s.aupd()
            if ido in (-1, 1):
                bx = s.slice(2).copy() if ido == 1 else None
                s.slice(1)[:] = c.op(s.slice(0).copy(), ido, bx)
            elif ido == 2:
                s.slice(1)[:] = c.bop(s.slice(0).copy())
            else:
                break
        print(name, "ref", int(g["iparam"][2]), int(g["nopx"]), "| rci", int(s.iparam[2]), int(s.iparam[8]),
              int(s.info[0]), flush=True)
        A, Mm = modes.dndrv5_pair(n)
        for method in (3, 2):
            G = pkg.DGen(dev(pkg, A), dev(pkg, Mm), mode, sigma, rtol=1e-13, maxit=5000, method=method)
            s = pkg.NsRci(n, 4, 20, "LM", 1e-10, bmat="G", mode=mode, mxiter=300, v0=g["v0"], device=True)
            s.aupd_gen(G)
            print(name, "device method", method, int(s.iparam[2]), int(s.iparam[8]), int(s.info[0]),
                  G.stats(), flush=True)


if __name__ == "__main__":
    main()
