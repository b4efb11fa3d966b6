"""Generate the committed golden fixtures from the REAL reference (oracle/_ref).

Run in the build container (where /root/reference exists):
    make -C oracle && python tests/golden/make_golden.py

Each fixture holds the inputs (operator spec, v0, parameters) and the reference's
outputs (Ritz values, iparam, stats, eigenvectors where small).  Matrices come
from oracle/matrices.py, which mirrors the device generators bit for bit.
"""
from __future__ import annotations

import ctypes as C
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import matrices as M  # noqa: E402
from oracle import ref  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def csr_op(rowptr, col, val):
    A = M.to_scipy(rowptr, col, val)
    return lambda x, *_: A @ x


def run_sym(name, mat, spec, nev, ncv, which, tol, mxiter=300, v0=None, keep_z=False, prec="d",
            **extra):
    rowptr, col, val = mat
    n = len(rowptr) - 1
    if v0 is None:
        v0, _ = M.dlarnv_uniform(n)
    if prec == "s":
        v0 = v0.astype(np.float32)
        extra["prec"] = "s"
    r = ref.dsaupd_solve(csr_op(rowptr, col, val), n, nev, ncv, which, tol, v0=v0,
                         mxiter=mxiter, return_state=True, prec=prec)
    assert r["info"] >= 0, r
    out = dict(spec=np.array(spec), nev=nev, ncv=ncv, which=np.array(which), tol=tol,
               mxiter=mxiter, v0=v0, info=r["info"], iparam=r["iparam"], d=r["d"],
               nopx=r["stats"]["nopx"], nrorth=r["stats"]["nrorth"],
               nitref=r["stats"]["nitref"], ritz=r["workl"][2 * ncv:3 * ncv],
               bounds=r["workl"][3 * ncv:4 * ncv], resid_norm=np.linalg.norm(r["resid"]))
    if keep_z:
        out["z"] = r["z"]
    out.update(extra)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, "info", r["info"], "iparam", r["iparam"][[2, 4, 8, 10]], "d", r["d"][:4], "...")
    return r


def run_ns(name, mat, spec, nev, ncv, which, tol, mxiter=300, v0=None, keep_z=False, prec="d",
           **extra):
    """dnaupd/dneupd fixture (SRC/dnaupd.f, SRC/dneupd.f); workl layout
    SRC/dnaupd.f:494-520 (ritzr at ih+ncv^2, ritzi, bounds)."""
    rowptr, col, val = mat
    n = len(rowptr) - 1
    if v0 is None:
        v0, _ = M.dlarnv_uniform(n)
    if prec == "s":
        v0 = v0.astype(np.float32)
        extra["prec"] = "s"
    r = ref.dnaupd_solve(csr_op(rowptr, col, val), n, nev, ncv, which, tol, v0=v0,
                         mxiter=mxiter, return_state=True, prec=prec)
    assert r["info"] >= 0, r
    o = ncv * ncv
    out = dict(spec=np.array(spec), nev=nev, ncv=ncv, which=np.array(which), tol=tol,
               mxiter=mxiter, v0=v0, info=r["info"], iparam=r["iparam"], dr=r["dr"], di=r["di"],
               nopx=r["stats"]["nopx"], nrorth=r["stats"]["nrorth"],
               nitref=r["stats"]["nitref"], ritzr=r["workl"][o:o + ncv],
               ritzi=r["workl"][o + ncv:o + 2 * ncv], bounds=r["workl"][o + 2 * ncv:o + 3 * ncv],
               eupd_info=r["eupd_info"])
    if keep_z:
        out["z"] = r["z"]
    out.update(extra)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, "info", r["info"], "iparam", r["iparam"][[2, 4, 8, 10]], "dr", r["dr"][:3],
          "di", r["di"][:3])
    return r


def nonsym_fixtures():
    cd10 = M.convdiff2d(10, 100.0)
    run_ns("n1_dnsimp", cd10, ["convdiff2d", 10, 100.0], 4, 20, "LM", 0.0, keep_z=True)
    run_ns("n2_dnsimp_tol", cd10, ["convdiff2d", 10, 100.0], 4, 20, "LM", 1e-10, keep_z=True)
    cd30 = M.convdiff2d(30, 100.0)
    run_ns("n3_convdiff_lm", cd30, ["convdiff2d", 30, 100.0], 10, 40, "LM", 1e-10, keep_z=True)
    run_ns("n4_convdiff_lr", cd10, ["convdiff2d", 10, 100.0], 4, 20, "LR", 1e-9, mxiter=3000)
    run_ns("n5_convdiff_li", cd10, ["convdiff2d", 10, 100.0], 4, 20, "LI", 1e-9, mxiter=3000)
    run_ns("n6_convdiff_sr", cd10, ["convdiff2d", 10, 100.0], 4, 20, "SR", 1e-9, mxiter=3000)
    cd100 = M.convdiff2d(100, 10.0)
    run_ns("n7_convdiff_real", cd100, ["convdiff2d", 100, 10.0], 10, 40, "LM", 1e-8,
           mxiter=3000)
    run_ns("n8_convdiff_capped", cd30, ["convdiff2d", 30, 100.0], 10, 40, "LM", 1e-14, mxiter=4)


def run_z(name, mat, spec, nev, ncv, which, tol, mxiter=300, mode=1, sigma=0j, keep_z=True,
          prec="z", **extra):
    """znaupd/zneupd fixture (SRC/znaupd.f, SRC/zneupd.f).  Mode 3 applies
    OP = inv(A - sigma I) with a sparse LU on the host, as a caller would."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spl
    rowptr, col, val = mat
    n = len(rowptr) - 1
    A = sp.csr_matrix((val, col, rowptr), shape=(n, n))
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)
    if prec == "c":
        v0 = v0.astype(np.complex64)
        extra["prec"] = "c"
    if mode == 1:
        op = lambda x, *_: A @ x  # noqa: E731
    else:
        lu = spl.splu((A - sigma * sp.identity(n, format="csr")).tocsc())
        op = lambda x, *_: lu.solve(x)  # noqa: E731
    r = ref.znaupd_solve(op, n, nev, ncv, which, tol, v0=v0, mxiter=mxiter, mode=mode,
                         sigma=sigma, return_state=True, prec=prec)
    assert r["info"] >= 0, r
    o = ncv * ncv
    out = dict(spec=np.array(spec), nev=nev, ncv=ncv, which=np.array(which), tol=tol,
               mxiter=mxiter, mode=mode, sigma=sigma, v0=v0, info=r["info"],
               iparam=r["iparam"], d=r["d"], ritz=r["workl"][o:o + ncv],
               bounds=r["workl"][o + ncv:o + 2 * ncv], eupd_info=r["eupd_info"])
    if keep_z:
        out["z"] = r["z"]
    out.update(extra)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, "info", r["info"], "iparam", r["iparam"][[2, 4, 8, 10]], "d", r["d"][:3])
    return r


def mode_fixtures():
    """Spectral-transformation modes (EXAMPLES/SYM/dsdrv2-6.f, NONSYM/dndrv2-3.f)
    with the caller operators of tests/modes.py."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import modes
    n = 400
    v0, _ = M.dlarnv_uniform(n)
    cases = [("m2_sym_std_si", "sym", modes.StdShiftInvert("fem1d", n, 0.0), 4, 20, "LM", 0.0),
             ("m3_sym_gen", "sym", modes.Caller("fem1d", 2, n), 4, 20, "LM", 0.0),
             ("m4_sym_gen_si", "sym", modes.Caller("fem1d", 3, n, 0.0), 4, 20, "LM", 0.0),
             ("m5_sym_buckling", "sym", modes.Caller("fem1d", 4, n, 1.0), 4, 20, "LM", 1.0),
             ("m6_sym_cayley", "sym", modes.Caller("fem1d", 5, n, 150.0), 4, 20, "LM", 150.0),
             ("m7_ns_std_si", "ns", modes.StdShiftInvert("convdiff1d", n, 1.0), 4, 20, "LM", 1.0),
             ("m8_ns_gen", "ns", modes.Caller("convdiff1d", 2, n), 4, 20, "LM", 0.0),
             ("m9_ns_gen_si", "ns", modes.Caller("convdiff1d", 3, n, 1.0), 4, 20, "LM", 1.0)]
    for name, fam, c, nev, ncv, which, sigma in cases:
        op = c.op
        if c.mode == 2:
            class Op:  # ref.dsaupd_solve reads op.ax for mode 2 (A*x written back over x)
                def __call__(self, x, k, bx):
                    return c.op(x, k, bx)

                @property
                def ax(self):
                    return c.ax
            op = Op()
        if fam == "sym":
            r = ref.dsaupd_solve(op, n, nev, ncv, which, 1e-10, v0=v0, mxiter=300, mode=c.mode,
                                 bmat=c.bmat, bop=c.bop, sigma=sigma)
            out = dict(d=r["d"], z=r["z"])
        else:
            r = ref.dnaupd_solve(op, n, nev, ncv, which, 1e-10, v0=v0, mxiter=300, mode=c.mode,
                                 bmat=c.bmat, bop=c.bop, sigmar=sigma)
            out = dict(dr=r["dr"], di=r["di"], z=r["z"])
        assert r["info"] >= 0 and r["eupd_info"] == 0, (name, r["info"], r.get("eupd_info"))
        np.savez_compressed(os.path.join(OUT, name + ".npz"), family=fam, mode=c.mode,
                            kind=np.array("fem1d" if "sym" in name else "convdiff1d"), n=n,
                            nev=nev, ncv=ncv, which=np.array(which), tol=1e-10, sigma=sigma,
                            v0=v0, info=r["info"], iparam=r["iparam"],
                            nopx=r["stats"]["nopx"], nbx=r["stats"]["nbx"], **out)
        print(name, "mode", c.mode, "iparam", r["iparam"][[2, 4, 8, 9, 10]],
              "d", out.get("d", out.get("dr"))[:4])


def complex_fixtures():
    run_z("z1_icb_zn", M.zdiag_icb(1000), ["zdiag_icb", 1000], 9, 19, "LM", 1e-6, mxiter=10000)
    zr = M.zrandom(2000, 20, 5, 100.0)
    run_z("z2_zrandom_lm", zr, ["zrandom", 2000, 20, 5, 100.0], 6, 20, "LM", 1e-10)
    run_z("z3_zrandom_si", zr, ["zrandom", 2000, 20, 5, 100.0], 6, 20, "LM", 1e-10, mode=3,
          sigma=0j)
    run_z("z4_zrandom_sr", zr, ["zrandom", 2000, 20, 5, 100.0], 5, 20, "SR", 1e-9, mxiter=3000)


def zmode_fixtures():
    """znaupd's generalized modes (EXAMPLES/COMPLEX/zndrv3.f mode 2, zndrv4.f
    mode 3: the 1-D convection-diffusion pair, n = 100, nev 4, ncv 20, LM),
    plus a complex rho with a complex shift, with the caller operators of
    tests/modes.py (sparse LU on the host, as the drivers' zgttrf/zgttrs)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import modes
    n = 100
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)
    cases = [("z5_zgen", 2, 0j, 10.0), ("z6_zgen_si", 3, 1 + 0j, 10.0),
             ("z7_zgen_si_complex", 3, 1 + 0.5j, 10 + 10j)]
    for name, mode, sigma, rho in cases:
        c = modes.ZCaller(mode, n, sigma, rho)
        r = ref.znaupd_solve(c.op, n, 4, 20, "LM", 1e-10, v0=v0, mxiter=300, mode=mode,
                             bmat="G", bop=c.bop, sigma=sigma, return_state=True)
        assert r["info"] >= 0 and r["eupd_info"] == 0, (name, r["info"], r.get("eupd_info"))
        o = 20 * 20
        np.savez_compressed(os.path.join(OUT, name + ".npz"), mode=mode, n=n, rho=complex(rho),
                            sigma=sigma, nev=4, ncv=20, which=np.array("LM"), tol=1e-10, v0=v0,
                            info=r["info"], iparam=r["iparam"], d=r["d"], z=r["z"],
                            ritz=r["workl"][o:o + 20], bounds=r["workl"][o + 20:o + 40])
        print(name, "mode", mode, "iparam", r["iparam"][[2, 4, 8, 9, 10]], "d", r["d"][:4])


def zndrv2_fixtures():
    """EXAMPLES/COMPLEX/zndrv2.f's operator (the 1-D convection-diffusion with
    1/h^2 scaling, rho = 10, n = 100) in shift-invert mode 3 -- the reference
    driver's zgttrf / zgttrs solve stands as the LU of run_z -- at its sigma = 0
    and at a complex shift."""
    n, rho = 100, 10.0
    h = 1.0 / (n + 1)
    s = rho / 2.0
    rows, cols, vals = [], [], []
    for i in range(n):
        for j, v in ((i - 1, -1.0 / h**2 - s / h), (i, 2.0 / h**2), (i + 1, -1.0 / h**2 + s / h)):
            if 0 <= j < n:
                rows.append(i)
                cols.append(j)
                vals.append(complex(v))
    rowptr = np.searchsorted(np.array(rows), np.arange(n + 1)).astype(np.int64)
    mat = (rowptr, np.array(cols, np.int32), np.array(vals, np.complex128))
    run_z("z8_zndrv2_si", mat, ["zndrv2", n, rho], 4, 20, "LM", 1e-10, mode=3, sigma=0j)
    run_z("z9_zndrv2_si_shift", mat, ["zndrv2", n, rho], 4, 20, "LM", 1e-10, mode=3,
          sigma=5000 + 2000j)


def cshift_fixtures():
    """dnaupd's complex shifts: EXAMPLES/NONSYM/dndrv5.f (mode 3, OP = Re
    inv[A - sigma M] M) and dndrv6.f's operator (Im ...) in mode 4, sigma =
    (0.4, 0.6), n = 100, nev 4, ncv 20, LM -- the drivers' zgttrf / zgttrs
    solve stands as a complex sparse LU (tests/modes.py CShiftCaller)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import modes
    n, sigma = 100, 0.4 + 0.6j
    v0, _ = M.dlarnv_uniform(n)
    for name, mode in (("m10_ns_cshift_re", 3), ("m11_ns_cshift_im", 4)):
        c = modes.CShiftCaller(mode, n, sigma)
        r = ref.dnaupd_solve(c.op, n, 4, 20, "LM", 1e-10, v0=v0, mxiter=300, mode=mode, bmat="G",
                             bop=c.bop, sigmar=sigma.real, sigmai=sigma.imag)
        assert r["info"] >= 0 and r["eupd_info"] == 0, (name, r["info"], r.get("eupd_info"))
        np.savez_compressed(os.path.join(OUT, name + ".npz"), family="ns", mode=mode,
                            kind=np.array("dndrv5"), n=n, nev=4, ncv=20, which=np.array("LM"),
                            tol=1e-10, sigmar=sigma.real, sigmai=sigma.imag, v0=v0,
                            info=r["info"], iparam=r["iparam"], nopx=r["stats"]["nopx"],
                            nbx=r["stats"]["nbx"], dr=r["dr"], di=r["di"], z=r["z"])
        print(name, "mode", mode, "iparam", r["iparam"][[2, 4, 8, 9, 10]], "dr", r["dr"][:4],
              "di", r["di"][:4])


def g7_dlarnv():
    lib = glob.glob(os.path.join(os.path.dirname(__import__("scipy").__file__), "..",
                                 "scipy.libs", "libscipy_openblas*.so"))[0]
    L = C.CDLL(lib)
    iseed = np.array([1, 3, 5, 7], np.int32)
    x = np.zeros(1000)
    L.scipy_dlarnv_(C.byref(C.c_int(2)), iseed.ctypes.data_as(C.POINTER(C.c_int)),
                    C.byref(C.c_int(1000)), x.ctypes.data_as(C.POINTER(C.c_double)))
    ours, seed = M.dlarnv_uniform(1000)
    assert np.array_equal(x, ours) and tuple(iseed) == tuple(seed), "dlarnv restatement drifted"
    np.savez_compressed(os.path.join(OUT, "g7_dlarnv.npz"), x=x, iseed_out=iseed,
                        iseed_in=np.array([1, 3, 5, 7], np.int32))
    print("g7_dlarnv ok, seed ->", iseed)


def g1_fresh_process_check():
    """info=0 in a fresh process == info=1 with the dlarnv(1,3,5,7) stream."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import numpy as np\nfrom oracle import ref, matrices as M\n"
            "A = M.to_scipy(*M.laplace2d(10, 121.0))\n"
            "r = ref.dsaupd_solve(lambda x,*_: A@x, 100, 4, 20, 'LM', 0.0)\n"
            "print(repr(r['d'].tolist()), int(r['iparam'][2]), int(r['iparam'][8]))" % ROOT)
    return ref.run_fresh(code)


def single_fixtures():
    """ssaupd/sseupd and snaupd/sneupd (SRC/ssaupd.f, SRC/snaupd.f): the reference's
    single-precision family on float32 arrays, OP = A @ x rounded to float32."""
    run_sym("s1_sssimp", M.laplace2d(10, 121.0), ["laplace2d", 10, 121.0], 4, 20, "LM", 0.0,
            keep_z=True, prec="s")
    run_sym("s2_icb_ss", M.diag(1000), ["diag", 1000], 9, 19, "LM", 1e-4, keep_z=True,
            mxiter=10000, prec="s")
    run_sym("s3_anderson3d", M.anderson(20, 3, 16.0, 1234), ["anderson", 20, 3, 16.0, 1234], 10,
            30, "LA", 1e-5, keep_z=True, prec="s")
    run_sym("s4_banded", M.banded_sym(20000, 1234, 512, 25), ["banded_sym", 20000, 1234, 512, 25],
            10, 30, "LA", 1e-5, keep_z=False, prec="s")
    run_ns("s5_bug1315_single", M.diag(1000), ["diag", 1000], 9, 19, "LM", 0.0, keep_z=True,
           mxiter=10000, prec="s")
    run_ns("s6_snsimp", M.convdiff2d(10, 10.0), ["convdiff2d", 10, 10.0], 4, 20, "LM", 1e-5,
           keep_z=True, prec="s")
    run_ns("s7_convdiff_lr", M.convdiff2d(30, 10.0), ["convdiff2d", 30, 10.0], 6, 30, "LR", 1e-5,
           keep_z=True, mxiter=3000, prec="s")
    # complex64 (cnaupd/cneupd; EXAMPLES/SIMPLE/cnsimp.f family)
    run_z("c1_icb_cn", M.zdiag_icb(1000), ["zdiag_icb", 1000], 9, 19, "LM", 1e-4, mxiter=10000,
          prec="c")
    zr = M.zrandom(2000, 20, 5, 100.0)
    run_z("c2_zrandom_lm", zr, ["zrandom", 2000, 20, 5, 100.0], 6, 20, "LM", 1e-5, prec="c")
    run_z("c3_zrandom_si", zr, ["zrandom", 2000, 20, 5, 100.0], 6, 20, "LM", 1e-5, mode=3,
          sigma=0j, prec="c")


if __name__ == "__main__":
    if sys.argv[1:] == ["s"]:
        single_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["ns"]:
        nonsym_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["modes"]:
        mode_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["z"]:
        complex_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["zmodes"]:
        zmode_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["zndrv2"]:
        zndrv2_fixtures()
        sys.exit(0)
    if sys.argv[1:] == ["cshift"]:
        cshift_fixtures()
        sys.exit(0)
    g7_dlarnv()
    r1 = run_sym("g1_dssimp", M.laplace2d(10, 121.0), ["laplace2d", 10, 121.0], 4, 20, "LM", 0.0,
                 keep_z=True)
    fresh = g1_fresh_process_check()
    assert fresh.strip() == "%r %d %d" % (r1["d"].tolist(), r1["iparam"][2], r1["iparam"][8]), fresh
    print("g1 fresh-process info=0 run identical to info=1 + dlarnv stream")
    run_sym("g2_icb_ds", M.diag(1000), ["diag", 1000], 9, 19, "LM", 1e-6, keep_z=True,
            mxiter=10000)
    run_sym("g3_anderson3d", M.anderson(20, 3, 16.0, 1234), ["anderson", 20, 3, 16.0, 1234], 10,
            30, "LA", 1e-10, keep_z=True)
    run_sym("g9_lap3d_degenerate", M.laplace3d(20), ["laplace3d", 20, 1.0], 10, 30, "LA", 1e-10,
            keep_z=False, degenerate=1)
    run_sym("g4_banded", M.banded_sym(20000, 1234, 512, 25), ["banded_sym", 20000, 1234, 512, 25],
            10, 30, "LA", 1e-8, keep_z=False)
    run_sym("g5_anderson2d_sa", M.anderson(40, 2, 4.0, 7), ["anderson", 40, 2, 4.0, 7], 6, 20,
            "SA", 1e-9, keep_z=False, mxiter=3000)
    run_sym("g6_anderson2d_be", M.anderson(40, 2, 4.0, 7), ["anderson", 40, 2, 4.0, 7], 6, 20,
            "BE", 1e-9, keep_z=False, mxiter=3000)
    run_sym("g10_anderson2d_sm", M.anderson(40, 2, 4.0, 7), ["anderson", 40, 2, 4.0, 7], 5, 24,
            "SM", 1e-8, keep_z=False, mxiter=3000)
    run_sym("g8_banded_capped", M.banded_sym(20000, 1234, 512, 25),
            ["banded_sym", 20000, 1234, 512, 25], 10, 30, "LA", 1e-14, mxiter=5)
    nonsym_fixtures()
    complex_fixtures()
    mode_fixtures()
    zmode_fixtures()
    zndrv2_fixtures()
    cshift_fixtures()
