"""ctypes driver for the REAL reference arpack-ng (oracle/_ref/libarpack_ref.so).

TEST INFRASTRUCTURE ONLY. Nothing in the product (`arpack-ng_amd/`) may import
this module; only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg use it, and only as the checker / the timed CPU baseline.

The library is built by `oracle/Makefile` from the reference's own Fortran
sources (SRC/*.f, UTIL/*.f, dbgini.f, staini.f) and the image's OpenBLAS. We
call the plain Fortran entry points, e.g. `dsaupd_` (SRC/dsaupd.f:182-186), with
every argument by reference plus the hidden trailing `size_t` lengths of the
CHARACTER dummies (bmat*1, which*2; howmny*1 for *eupd) — the gfortran/flang
ABI the ICB wrappers (SRC/icbads.F90:3-35) themselves rely on.

The driver owns the RCI loop exactly like the reference's callers
(TESTS/icb_arpack_c.c:60-75, EXAMPLES/SIMPLE/dssimp.f:293-326): it services
ido=-1/1 with the user OP (a Python callable y = op(x)) and, for bmat='G',
ido=2 with B.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_ref", "libarpack_ref.so")
CSR_OMP_PATH = os.path.join(_HERE, "_ref", "libcsr_omp.so")

_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def build(quiet: bool = True) -> bool:
    """Build oracle/_ref from /root/reference (only possible where it exists)."""
    if not os.path.isdir("/root/reference"):
        return available()
    r = subprocess.run(["make", "-C", _HERE, "-j8"], capture_output=quiet, text=True)
    return r.returncode == 0 and available()


def lib():
    global _lib
    if _lib is None:
        if not available():
            raise RuntimeError("oracle/_ref/libarpack_ref.so missing: run `make -C oracle`")
        _lib = C.CDLL(LIB_PATH)
    return _lib


_i = C.POINTER(C.c_int)
_d = C.POINTER(C.c_double)


def _pi(a):
    return a.ctypes.data_as(_i)


def _pd(a):
    return a.ctypes.data_as(C.c_void_p)  # double* or float* (untyped Fortran entry)


def _ci(x):
    return C.byref(C.c_int(int(x)))


class Timing(C.Structure):
    """The /timing/ common block of stat.h:8-21 (integers first, then reals)."""
    _fields_ = [("nopx", C.c_int), ("nbx", C.c_int), ("nrorth", C.c_int),
                ("nitref", C.c_int), ("nrstrt", C.c_int)] + \
               [(nm, C.c_float) for nm in (
                   "tsaupd", "tsaup2", "tsaitr", "tseigt", "tsgets", "tsapps", "tsconv",
                   "tnaupd", "tnaup2", "tnaitr", "tneigh", "tngets", "tnapps", "tnconv",
                   "tcaupd", "tcaup2", "tcaitr", "tceigh", "tcgets", "tcapps", "tcconv",
                   "tmvopx", "tmvbx", "tgetv0", "titref", "trvec")]


def timing() -> Timing:
    return Timing.in_dll(lib(), "timing_")


def dsaupd_solve(op, n, nev, ncv, which="LM", tol=0.0, v0=None, mxiter=300,
                 mode=1, bmat="I", bop=None, rvec=True, sigma=0.0, ishift=1,
                 shifts=None, return_state=False, prec="d", howmny="A"):
    """Run dsaupd_/dseupd_ to completion. Returns dict with d, z, iparam, info...

    `op(x, ido, bx)` computes OP*x (bx = B*x slice for modes 3-5, else None);
    `bop(x)` computes B*x when bmat='G'.  prec="s": ssaupd_/sseupd_ (SRC/ssaupd.f)
    on float32 arrays.
    """
    L = lib()
    dt = np.float32 if prec == "s" else np.float64
    ct = C.c_float if prec == "s" else C.c_double
    ido = np.zeros(1, np.int32)
    info = np.zeros(1, np.int32)
    resid = np.zeros(n, dt) if v0 is None else np.array(v0, dtype=dt, copy=True)
    info[0] = 0 if v0 is None else 1
    ldv = n
    v = np.asfortranarray(np.zeros((ldv, ncv), dt))
    iparam = np.zeros(11, np.int32)
    ipntr = np.zeros(11, np.int32)
    iparam[0] = ishift
    iparam[2] = mxiter
    iparam[6] = mode
    workd = np.zeros(3 * n, dt)
    lworkl = ncv * ncv + 8 * ncv
    workl = np.zeros(lworkl, dt)
    tolc = ct(tol)
    bm = bmat.encode()
    wh = which.encode()
    n_rci = 0
    while True:
        getattr(L, prec + "saupd_")(_pi(ido), C.c_char_p(bm), _ci(n), C.c_char_p(wh), _ci(nev), C.byref(tolc),
                  _pd(resid), _ci(ncv), _pd(v), _ci(ldv), _pi(iparam), _pi(ipntr),
                  _pd(workd), _pd(workl), _ci(lworkl), _pi(info),
                  C.c_size_t(1), C.c_size_t(2))
        n_rci += 1
        k = int(ido[0])
        if k in (-1, 1):
            x = workd[ipntr[0] - 1: ipntr[0] - 1 + n]
            bx = workd[ipntr[2] - 1: ipntr[2] - 1 + n] if (mode >= 3 and k == 1) else None
            y = op(x.copy(), k, None if bx is None else bx.copy())
            workd[ipntr[1] - 1: ipntr[1] - 1 + n] = y
            if mode == 2:  # user overwrites x with A*x (EXAMPLES/SYM/dsdrv3.f)
                workd[ipntr[0] - 1: ipntr[0] - 1 + n] = op.ax  # type: ignore[attr-defined]
        elif k == 2:
            x = workd[ipntr[0] - 1: ipntr[0] - 1 + n]
            workd[ipntr[1] - 1: ipntr[1] - 1 + n] = bop(x.copy())
        elif k == 3:
            np_ = int(iparam[7])
            workl[ipntr[10] - 1: ipntr[10] - 1 + np_] = shifts(np_)
        else:
            break
    out = dict(info=int(info[0]), iparam=iparam.copy(), ipntr=ipntr.copy(), n_rci=n_rci,
               tol=tolc.value)
    st = timing()
    out["stats"] = dict(nopx=st.nopx, nbx=st.nbx, nrorth=st.nrorth, nitref=st.nitref,
                        nrstrt=st.nrstrt)
    if return_state:
        out.update(resid=resid.copy(), v=v.copy(), workl=workl.copy(), workd=workd.copy())
    if info[0] < 0:
        return out
    nconv = int(iparam[4])
    d = np.zeros(nev, dt)
    z = np.asfortranarray(np.zeros((n, nev), dt))
    select = np.zeros(ncv, np.int32)
    ierr = np.zeros(1, np.int32)
    getattr(L, prec + "seupd_")(_ci(1 if rvec else 0), C.c_char_p(howmny.encode()), _pi(select), _pd(d),
              _pd(z), _ci(n), C.byref(ct(sigma)), C.c_char_p(bm), _ci(n), C.c_char_p(wh), _ci(nev),
              C.byref(tolc), _pd(resid), _ci(ncv), _pd(v), _ci(ldv), _pi(iparam), _pi(ipntr),
              _pd(workd), _pd(workl), _ci(lworkl), _pi(ierr),
              C.c_size_t(1), C.c_size_t(1), C.c_size_t(2))
    out.update(eupd_info=int(ierr[0]), d=d[:nconv].copy(), z=z[:, :nconv].copy(), nconv=nconv,
               workl_after=workl.copy())
    return out


def dnaupd_solve(op, n, nev, ncv, which="LM", tol=0.0, v0=None, mxiter=300, mode=1,
                 bmat="I", bop=None, rvec=True, sigmar=0.0, sigmai=0.0, return_state=False,
                 prec="d", ishift=1, shifts=None):
    """Run dnaupd_/dneupd_ (SRC/dnaupd.f:406, SRC/dneupd.f) to completion
    (prec="s": snaupd_/sneupd_ on float32 arrays)."""
    L = lib()
    dt = np.float32 if prec == "s" else np.float64
    ct = C.c_float if prec == "s" else C.c_double
    ido = np.zeros(1, np.int32)
    info = np.zeros(1, np.int32)
    resid = np.zeros(n, dt) if v0 is None else np.array(v0, dtype=dt, copy=True)
    info[0] = 0 if v0 is None else 1
    ldv = n
    v = np.asfortranarray(np.zeros((ldv, ncv), dt))
    iparam = np.zeros(11, np.int32)
    ipntr = np.zeros(14, np.int32)
    iparam[0] = ishift
    iparam[2] = mxiter
    iparam[6] = mode
    workd = np.zeros(3 * n, dt)
    lworkl = 3 * ncv * ncv + 6 * ncv
    workl = np.zeros(lworkl, dt)
    tolc = ct(tol)
    bm = bmat.encode()
    wh = which.encode()
    while True:
        getattr(L, prec + "naupd_")(_pi(ido), C.c_char_p(bm), _ci(n), C.c_char_p(wh), _ci(nev), C.byref(tolc),
                  _pd(resid), _ci(ncv), _pd(v), _ci(ldv), _pi(iparam), _pi(ipntr),
                  _pd(workd), _pd(workl), _ci(lworkl), _pi(info),
                  C.c_size_t(1), C.c_size_t(2))
        k = int(ido[0])
        if k in (-1, 1):
            x = workd[ipntr[0] - 1: ipntr[0] - 1 + n]
            workd[ipntr[1] - 1: ipntr[1] - 1 + n] = op(x.copy(), k, None)
        elif k == 2:
            x = workd[ipntr[0] - 1: ipntr[0] - 1 + n]
            workd[ipntr[1] - 1: ipntr[1] - 1 + n] = bop(x.copy())
        elif k == 3:  # user shifts: real parts at ipntr(14), imaginary parts np later
            np_ = int(iparam[7])
            re, im = shifts(np_)
            o = int(ipntr[13]) - 1
            workl[o:o + np_] = re
            workl[o + np_:o + 2 * np_] = im
        else:
            break
    out = dict(info=int(info[0]), iparam=iparam.copy(), ipntr=ipntr.copy(), tol=tolc.value)
    st = timing()
    out["stats"] = dict(nopx=st.nopx, nbx=st.nbx, nrorth=st.nrorth, nitref=st.nitref,
                        nrstrt=st.nrstrt)
    if return_state:
        out.update(resid=resid.copy(), v=v.copy(), workl=workl.copy())
    if info[0] < 0:
        return out
    nconv = int(iparam[4])
    dr = np.zeros(nev + 1, dt)
    di = np.zeros(nev + 1, dt)
    z = np.asfortranarray(np.zeros((n, nev + 1), dt))
    select = np.zeros(ncv, np.int32)
    workev = np.zeros(3 * ncv, dt)
    ierr = np.zeros(1, np.int32)
    getattr(L, prec + "neupd_")(_ci(1 if rvec else 0), C.c_char_p(b"A"), _pi(select), _pd(dr),
              _pd(di), _pd(z), _ci(n), C.byref(ct(sigmar)), C.byref(ct(sigmai)), _pd(workev),
              C.c_char_p(bm), _ci(n), C.c_char_p(wh), _ci(nev), C.byref(tolc), _pd(resid),
              _ci(ncv), _pd(v), _ci(ldv), _pi(iparam), _pi(ipntr), _pd(workd), _pd(workl),
              _ci(lworkl), _pi(ierr), C.c_size_t(1), C.c_size_t(1), C.c_size_t(2))
    out.update(eupd_info=int(ierr[0]), dr=dr[:nconv].copy(), di=di[:nconv].copy(),
               z=z[:, :nconv].copy(), nconv=nconv)
    return out


def znaupd_solve(op, n, nev, ncv, which="LM", tol=0.0, v0=None, mxiter=300, mode=1,
                 bmat="I", bop=None, rvec=True, sigma=0.0 + 0.0j, return_state=False,
                 prec="z"):
    """Run znaupd_/zneupd_ (SRC/znaupd.f, SRC/zneupd.f) to completion
    (prec="c": cnaupd_/cneupd_ on complex64 arrays)."""
    L = lib()
    ct = np.complex64 if prec == "c" else np.complex128
    rt = np.float32 if prec == "c" else np.float64
    ido = np.zeros(1, np.int32)
    info = np.zeros(1, np.int32)
    resid = np.zeros(n, ct) if v0 is None else np.array(v0, dtype=ct, copy=True)
    info[0] = 0 if v0 is None else 1
    ldv = n
    v = np.asfortranarray(np.zeros((ldv, ncv), ct))
    iparam = np.zeros(11, np.int32)
    ipntr = np.zeros(14, np.int32)
    iparam[0] = 1
    iparam[2] = mxiter
    iparam[6] = mode
    workd = np.zeros(3 * n, ct)
    lworkl = 3 * ncv * ncv + 5 * ncv
    workl = np.zeros(lworkl, ct)
    rwork = np.zeros(ncv, rt)
    tolc = (C.c_float if prec == "c" else C.c_double)(tol)
    bm = bmat.encode()
    wh = which.encode()
    while True:
        getattr(L, prec + "naupd_")(_pi(ido), C.c_char_p(bm), _ci(n), C.c_char_p(wh), _ci(nev), C.byref(tolc),
                  _pd(resid), _ci(ncv), _pd(v), _ci(ldv), _pi(iparam), _pi(ipntr),
                  _pd(workd), _pd(workl), _ci(lworkl), _pd(rwork), _pi(info),
                  C.c_size_t(1), C.c_size_t(2))
        k = int(ido[0])
        if k in (-1, 1):
            x = workd[ipntr[0] - 1: ipntr[0] - 1 + n]
            bx = workd[ipntr[2] - 1: ipntr[2] - 1 + n] if (mode >= 3 and k == 1) else None
            workd[ipntr[1] - 1: ipntr[1] - 1 + n] = op(x.copy(), k,
                                                       None if bx is None else bx.copy())
        elif k == 2:
            x = workd[ipntr[0] - 1: ipntr[0] - 1 + n]
            workd[ipntr[1] - 1: ipntr[1] - 1 + n] = bop(x.copy())
        elif k == 3:  # user shifts: real parts at ipntr(14), imaginary parts np later
            np_ = int(iparam[7])
            re, im = shifts(np_)
            o = int(ipntr[13]) - 1
            workl[o:o + np_] = re
            workl[o + np_:o + 2 * np_] = im
        else:
            break
    out = dict(info=int(info[0]), iparam=iparam.copy(), ipntr=ipntr.copy(), tol=tolc.value)
    if return_state:
        out.update(resid=resid.copy(), v=v.copy(), workl=workl.copy())
    if info[0] < 0:
        return out
    nconv = int(iparam[4])
    d = np.zeros(nev + 1, ct)
    z = np.asfortranarray(np.zeros((n, nev), ct))
    select = np.zeros(ncv, np.int32)
    workev = np.zeros(2 * ncv, ct)
    ierr = np.zeros(1, np.int32)
    sg = np.array([sigma], ct)
    getattr(L, prec + "neupd_")(_ci(1 if rvec else 0), C.c_char_p(b"A"), _pi(select), _pd(d), _pd(z), _ci(n),
              _pd(sg), _pd(workev), C.c_char_p(bm), _ci(n), C.c_char_p(wh), _ci(nev),
              C.byref(tolc), _pd(resid), _ci(ncv), _pd(v), _ci(ldv), _pi(iparam), _pi(ipntr),
              _pd(workd), _pd(workl), _ci(lworkl), _pd(rwork), _pi(ierr),
              C.c_size_t(1), C.c_size_t(1), C.c_size_t(2))
    out.update(eupd_info=int(ierr[0]), d=d[:nconv].copy(), z=z[:, :nconv].copy(), nconv=nconv)
    return out


def run_fresh(code: str) -> str:
    """Run `code` in a fresh interpreter (the reference's dgetv0 seed is a
    process-wide SAVE variable initialised once, SRC/dgetv0.f:202-208)."""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       cwd=os.path.dirname(_HERE))
    if r.returncode != 0:
        raise RuntimeError(r.stderr)
    return r.stdout


# ---- multithreaded CSR SpMV (user OP of the CPU baseline) ------------------------------

_csr = None


def csr_omp():
    global _csr
    if _csr is None:
        _csr = C.CDLL(CSR_OMP_PATH)
        for f in (_csr.csr_spmv_f64, _csr.csr_spmv_c128):
            f.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                          C.c_void_p, C.c_int]
    return _csr


def csr_matvec(rowptr64, col32, val, nthreads=0):
    """Return op(x) -> A x using the OpenMP CSR kernel (fp64)."""
    lib_ = csr_omp()
    n = len(rowptr64) - 1
    y = np.empty(n)

    def op(x, *_):
        x = np.ascontiguousarray(x)
        lib_.csr_spmv_f64(n, rowptr64.ctypes.data, col32.ctypes.data, val.ctypes.data,
                          x.ctypes.data, y.ctypes.data, nthreads)
        return y.copy()
    return op


def csr_matvec_c128(rowptr64, col32, val, nthreads=0):
    """Return op(x) -> A x using the OpenMP CSR kernel (complex128, interleaved)."""
    lib_ = csr_omp()
    n = len(rowptr64) - 1
    vv = np.ascontiguousarray(val, np.complex128)
    y = np.empty(n, np.complex128)

    def op(x, *_):
        x = np.ascontiguousarray(x, np.complex128)
        lib_.csr_spmv_c128(n, rowptr64.ctypes.data, col32.ctypes.data, vv.ctypes.data,
                           x.ctypes.data, y.ctypes.data, nthreads)
        return y.copy()
    return op
