import sys, os, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from conftest import load_pkg, GOLDEN
from test_gpu_parity import _mat
pkg = load_pkg()
for name in ["g1_dssimp","g2_icb_ds","g3_anderson3d","g4_banded","g5_anderson2d_sa","g6_anderson2d_be","g8_banded_capped","g9_lap3d_degenerate","g10_anderson2d_sm"]:
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    rp, col, val = _mat(g["spec"])
    A = pkg.CSR.from_arrays(rp, col, val)
    d, z, res = pkg.eigsh(A, len(rp)-1, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), v0=g["v0"], mxiter=int(g["mxiter"]), device=True)
    print(name, res, pkg.stats(), "ref iparam", g["iparam"][[2,4,8,10]])
