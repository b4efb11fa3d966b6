"""GPU: dseupd's own error codes (SRC/dseupd.f:125-148) equal the reference's
after the same dsaupd run: HOWMNY not 'A'/'P'/'S' with RVEC (-15), HOWMNY = 'S'
(-16, "not yet implemented"); and the reference's quick return when nothing
converged (SRC/dseupd.f:312 jumps out with info = 0 before the -14 test, which
therefore never fires for nconv = 0) is reproduced too.  The reference runs through oracle/_ref (Fortran ABI),
this library through dsaupd_c/dseupd_c with the caller's OP on host arrays."""
import numpy as np
import pytest

from oracle import matrices as M
from oracle import ref

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built")]


@pytest.mark.parametrize("howmny,mxiter,tol,m,nev,ncv", [("X", 300, 1e-8, 10, 4, 20),
                                                        ("S", 300, 1e-8, 10, 4, 20),
                                                        ("A", 1, 1e-15, 30, 6, 14)])
def test_dseupd_error_codes(pkg, howmny, mxiter, tol, m, nev, ncv):
    rp, col, val = M.laplace2d(m, float((m + 1) ** 2))  # EXAMPLES/SIMPLE/dssimp.f's operator
    A = M.to_scipy(rp, col, val)
    n = m * m
    v0 = M.dlarnv_uniform(n)[0]
    want = ref.dsaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LM", tol, v0=v0, mxiter=mxiter,
                            howmny=howmny)
    s = pkg.SymRci(n, nev, ncv, "LM", tol, mxiter=mxiter, v0=v0)
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        else:
            break
    assert int(s.info[0]) == want["info"] and int(s.iparam[4]) == int(want["iparam"][4])
    if want["eupd_info"] == 0:  # nconv = 0: the quick return
        assert int(want["iparam"][4]) == 0
        d, z, nconv = s.eupd(rvec=True, howmny=howmny)
        assert nconv == 0 and len(d) == 0
        return
    with pytest.raises(pkg.ArpackError) as e:
        s.eupd(rvec=True, howmny=howmny)
    assert e.value.info == want["eupd_info"]
