"""CPU: the *aupd argument checks return the reference's error codes.

SRC/dsaupd.f:501-543, SRC/dnaupd.f:500-524, SRC/znaupd.f:474-500: each check
assigns `ierr` in a fixed order (dsaupd: the -4 .. -7 tests are independent IFs
after the -1/-2/-3 chain, so a later failing test overrides an earlier one;
dnaupd/znaupd: one ELSE-IF chain).  The codes come back in `info` with
ido = 99 before any work is done, so no GPU is touched.  Every case is run
through the real reference (oracle/_ref, Fortran ABI) and through this
library's ICB (`*_c`) and Fortran (`*_`) entry points.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import ref

pytestmark = pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built")

_P = C.c_void_p
_I = C.POINTER(C.c_int)


def _ip(a):
    return a.ctypes.data_as(_I)


def _fresh(path):
    """A separate CDLL handle: its function objects carry no argtypes from the
    package's or the oracle's own declarations."""
    return C.CDLL(path)


BASE_S = dict(n=100, nev=4, ncv=20, which="LM", bmat="I", mode=1, ishift=1, mxiter=300, lw=None)
BASE_N = dict(n=100, nev=4, ncv=20, which="LM", bmat="I", mode=1, ishift=1, mxiter=300, lw=None)

CASES_S = [dict(n=0), dict(nev=0), dict(ncv=4), dict(ncv=101, n=100), dict(mxiter=0),
           dict(which="LR"), dict(which="XX"), dict(bmat="X"), dict(lw=100), dict(mode=6),
           dict(mode=0), dict(mode=1, bmat="G"), dict(ishift=2), dict(ishift=-1),
           dict(nev=1, which="BE"),
           # combined failures: the reference's check order decides
           dict(n=0, mxiter=0), dict(nev=0, bmat="X"), dict(ncv=4, lw=10), dict(mxiter=0, which="XX"),
           dict(bmat="X", mode=6), dict(mode=6, ishift=2), dict(n=0, mode=9), dict(lw=1, ishift=5)]
CASES_N = [dict(n=0), dict(nev=0), dict(ncv=5), dict(ncv=101, n=100), dict(mxiter=0),
           dict(which="LA"), dict(which="BE"), dict(bmat="X"), dict(lw=100), dict(mode=5),
           dict(mode=0), dict(mode=1, bmat="G"), dict(ishift=2),
           dict(n=0, mxiter=0), dict(mxiter=0, which="XX"), dict(bmat="X", lw=1),
           dict(mode=5, ishift=3), dict(lw=1, mode=7)]
# znaupd: ncv > nev suffices, modes 1-3, no ishift test (SRC/znaupd.f:474-498)
CASES_Z = [dict(n=0), dict(nev=0), dict(ncv=4), dict(ncv=101, n=100), dict(mxiter=0),
           dict(which="LA"), dict(which="BE"), dict(bmat="X"), dict(lw=100), dict(mode=4),
           dict(mode=0), dict(mode=1, bmat="G"),
           dict(n=0, mxiter=0), dict(mxiter=0, which="XX"), dict(bmat="X", lw=1), dict(lw=1, mode=7)]


def _args(base, over, lw_of):
    a = dict(base)
    a.update(over)
    if a["lw"] is None:
        a["lw"] = lw_of(a["ncv"])
    return a


def _arrays(a, cplx=False, single=False):
    dt = ((np.complex64 if single else np.complex128) if cplx else
          (np.float32 if single else np.float64))
    n, ncv = max(a["n"], 1), max(a["ncv"], 1)
    return dict(resid=np.zeros(n, dt), v=np.zeros((ncv, n), dt), workd=np.zeros(3 * n, dt),
                workl=np.zeros(max(a["lw"], 1), dt),
                rwork=np.zeros(ncv, np.float32 if single else np.float64),
                ipntr=np.zeros(14, np.int32))


def _iparam(a):
    ip = np.zeros(11, np.int32)
    ip[0], ip[2], ip[6] = a["ishift"], a["mxiter"], a["mode"]
    return ip


def _call_fortran(L, name, a, cplx=False, single=False):
    """name_(ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
    workl, lworkl, [rwork,] info, len(bmat), len(which)) -- every argument by reference."""
    ar = _arrays(a, cplx, single)
    ido, info = np.zeros(1, np.int32), np.zeros(1, np.int32)
    ip = _iparam(a)
    n, nev, ncv, ldv, lw = (np.array([x], np.int32) for x in (a["n"], a["nev"], a["ncv"],
                                                               max(a["n"], 1), a["lw"]))
    tol = np.zeros(1, np.float32 if single else np.float64)
    f = getattr(L, name)
    f.restype = None
    args = [_ip(ido), a["bmat"].encode(), _ip(n), a["which"].encode(), _ip(nev), _P(tol.ctypes.data),
            _P(ar["resid"].ctypes.data), _ip(ncv), _P(ar["v"].ctypes.data), _ip(ldv), _ip(ip),
            _ip(ar["ipntr"]), _P(ar["workd"].ctypes.data), _P(ar["workl"].ctypes.data), _ip(lw)]
    if cplx:
        args.append(_P(ar["rwork"].ctypes.data))
    args += [_ip(info), C.c_size_t(1), C.c_size_t(2)]
    f(*args)
    return int(ido[0]), int(info[0])


def _call_icb(L, name, a, cplx=False, single=False):
    """name_c(int* ido, char* bmat, int n, char* which, int nev, double tol, resid, int ncv,
    v, int ldv, iparam, ipntr, workd, workl, int lworkl, [rwork,] int* info)  (ICB/arpack.h)"""
    ar = _arrays(a, cplx, single)
    ido, info = np.zeros(1, np.int32), np.zeros(1, np.int32)
    ip = _iparam(a)
    f = getattr(L, name)
    args = [_ip(ido), a["bmat"].encode(), C.c_int(a["n"]), a["which"].encode(), C.c_int(a["nev"]),
            C.c_float(0.0) if single else C.c_double(0.0), _P(ar["resid"].ctypes.data), C.c_int(a["ncv"]), _P(ar["v"].ctypes.data),
            C.c_int(max(a["n"], 1)), _ip(ip), _ip(ar["ipntr"]), _P(ar["workd"].ctypes.data),
            _P(ar["workl"].ctypes.data), C.c_int(a["lw"])]
    if cplx:
        args.append(_P(ar["rwork"].ctypes.data))
    args.append(_ip(info))
    f.restype = None
    f(*args)
    return int(ido[0]), int(info[0])


@pytest.mark.parametrize("over", CASES_S)
def test_dsaupd_error_codes(pkg, over):
    a = _args(BASE_S, over, lambda ncv: ncv * ncv + 8 * ncv)
    want = _call_fortran(_fresh(ref.LIB_PATH), "dsaupd_", a)
    assert want[0] == 99 and want[1] < 0, want
    assert _call_icb(_fresh(pkg.LIB_PATH), "dsaupd_c", a) == want
    assert _call_fortran(_fresh(pkg.LIB_PATH), "dsaupd_", a) == want


@pytest.mark.parametrize("over", CASES_N)
def test_dnaupd_error_codes(pkg, over):
    a = _args(BASE_N, over, lambda ncv: 3 * ncv * ncv + 6 * ncv)
    want = _call_fortran(_fresh(ref.LIB_PATH), "dnaupd_", a)
    assert want[0] == 99 and want[1] < 0, want
    assert _call_icb(_fresh(pkg.LIB_PATH), "dnaupd_c", a) == want
    assert _call_fortran(_fresh(pkg.LIB_PATH), "dnaupd_", a) == want


@pytest.mark.parametrize("over", CASES_Z)
def test_znaupd_error_codes(pkg, over):
    a = _args(BASE_N, over, lambda ncv: 3 * ncv * ncv + 5 * ncv)
    want = _call_fortran(_fresh(ref.LIB_PATH), "znaupd_", a, cplx=True)
    assert want[0] == 99 and want[1] < 0, want
    assert _call_icb(_fresh(pkg.LIB_PATH), "znaupd_c", a, cplx=True) == want
    assert _call_fortran(_fresh(pkg.LIB_PATH), "znaupd_", a, cplx=True) == want


@pytest.mark.parametrize("fam,cases", [("s", CASES_S), ("n", CASES_N), ("z", CASES_Z)])
def test_single_precision_error_codes(pkg, fam, cases):
    """ssaupd / snaupd / cnaupd: same checks as the double families (SRC/ssaupd.f,
    snaupd.f, cnaupd.f), float arguments (ICB: float tol by value)."""
    name, lw_of, cplx = {"s": ("ssaupd", lambda c: c * c + 8 * c, False),
                         "n": ("snaupd", lambda c: 3 * c * c + 6 * c, False),
                         "z": ("cnaupd", lambda c: 3 * c * c + 5 * c, True)}[fam]
    for over in cases:
        a = _args(BASE_S, over, lw_of)
        want = _call_fortran(_fresh(ref.LIB_PATH), name + "_", a, cplx, True)
        assert want[0] == 99 and want[1] < 0, (over, want)
        assert _call_icb(_fresh(pkg.LIB_PATH), name + "_c", a, cplx, True) == want, over
        assert _call_fortran(_fresh(pkg.LIB_PATH), name + "_", a, cplx, True) == want, over


@pytest.mark.parametrize("name,cplx,lw_of", [
    ("dsaupd_c", False, lambda ncv: ncv * ncv + 8 * ncv),
    ("dnaupd_c", False, lambda ncv: 3 * ncv * ncv + 6 * ncv),
    ("znaupd_c", True, lambda ncv: 3 * ncv * ncv + 5 * ncv)])
def test_ncv_above_engine_limit(pkg, name, cplx, lw_of):
    """ncv above the engine's documented limit (8000: the finalize stages ncv + 2
    sums in 64 KB of LDS) is rejected like ncv > n, info = -3,
    before any array is touched (the arrays here are untouched lazy zero pages)."""
    a = dict(BASE_S if name[1] == "s" else BASE_N, n=9000, ncv=8001, nev=4)
    a["lw"] = lw_of(a["ncv"])
    assert _call_icb(_fresh(pkg.LIB_PATH), name, a, cplx=cplx) == (99, -3)
    a["ncv"] = 8000  # at the limit the checks pass (-7 from a short workl proves it)
    a["lw"] = 1
    assert _call_icb(_fresh(pkg.LIB_PATH), name, a, cplx=cplx) == (99, -7)
