"""GPU: user-supplied shifts (iparam(1) = ishift = 0): *aupd returns ido = 3
with iparam(8) = np and the caller writes np shifts at workl(ipntr(11))
(SRC/dsaupd.f:90-96, SRC/dsaup2.f:536-560; SRC/dnaupd.f for the real and
imaginary parts).  The same fixed shifts go to the reference and to this
library; restart counts, OP*x counts and Ritz values must agree."""
import numpy as np
import pytest

from oracle import matrices as M
from oracle import ref

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built")]


def _shifts(lo, hi):
    return lambda np_: np.linspace(lo, hi, np_)


@pytest.mark.parametrize("which,lo,hi", [("LM", 20.0, 500.0), ("SM", 300.0, 900.0)])
def test_dsaupd_user_shifts(pkg, which, lo, hi):
    m = 10
    rp, col, val = M.laplace2d(m, float((m + 1) ** 2))   # dssimp's operator, spectrum (0, 968)
    A = M.to_scipy(rp, col, val)
    n, nev, ncv, tol = m * m, 4, 20, 1e-8
    v0 = M.dlarnv_uniform(n)[0]
    sh = _shifts(lo, hi)
    want = ref.dsaupd_solve(lambda x, *_: A @ x, n, nev, ncv, which, tol, v0=v0, mxiter=300,
                            ishift=0, shifts=sh)
    s = pkg.SymRci(n, nev, ncv, which, tol, mxiter=300, ishift=0, v0=v0)
    n3 = 0
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        elif ido == 3:
            k = int(s.iparam[7])
            o = int(s.ipntr[10]) - 1
            s.workl[o:o + k] = sh(k)
            n3 += 1
        else:
            break
    assert n3 > 0
    assert int(s.info[0]) == want["info"]
    assert int(s.iparam[2]) == int(want["iparam"][2])      # restart cycles
    assert int(s.iparam[8]) == int(want["iparam"][8])      # OP*x
    d, z, nconv = s.eupd()
    assert nconv == want["nconv"]
    np.testing.assert_allclose(np.sort(d), np.sort(want["d"]), rtol=1e-9)


def test_dnaupd_user_shifts(pkg):
    """dnaupd: real and imaginary parts of the shifts at workl(ipntr(14)) and
    np entries later (SRC/dnaupd.f, remark 5); real shifts inside the
    unwanted part of a convection-diffusion spectrum, which='LM'."""
    m = 12
    rp, col, val = M.convdiff2d(m, 10.0)
    A = M.to_scipy(rp, col, val)
    n, nev, ncv, tol = m * m, 4, 20, 1e-8
    v0 = M.dlarnv_uniform(n)[0]
    lam = np.linalg.eigvals(A.toarray())
    lo, hi = np.abs(lam).min(), np.sort(np.abs(lam))[-3 * nev]
    sh = lambda k: (np.linspace(lo, hi, k), np.zeros(k))  # noqa: E731
    want = ref.dnaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LM", tol, v0=v0, mxiter=300,
                            ishift=0, shifts=sh)
    s = pkg.NsRci(n, nev, ncv, "LM", tol, mxiter=300, ishift=0, v0=v0)
    n3 = 0
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        elif ido == 3:
            k = int(s.iparam[7])
            o = int(s.ipntr[13]) - 1
            re, im = sh(k)
            s.workl[o:o + k] = re
            s.workl[o + k:o + 2 * k] = im
            n3 += 1
        else:
            break
    assert n3 > 0
    assert int(s.info[0]) == want["info"]
    assert int(s.iparam[2]) == int(want["iparam"][2])
    assert int(s.iparam[8]) == int(want["iparam"][8])
    dr, di, z, nconv = s.eupd()
    assert nconv == want["nconv"]
    got = np.sort_complex(dr[:nconv] + 1j * di[:nconv])
    ref_ = np.sort_complex(want["dr"] + 1j * want["di"])
    np.testing.assert_allclose(got, ref_, rtol=1e-8)
