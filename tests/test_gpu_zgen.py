"""GPU: znaupd's generalized modes (bmat = 'G', modes 2-3; SRC/znaupd.f:23-31)
free-running on the device (arpack_hip_znaupd_gen, VERDICT r05 missing #4's
complex half): OP*x and B*x served by the device operator pair (complex CSR
products, the inverse by the device BiCGStab on C = A - sigma M), against the
reference fixtures z5-z7 the reference made with the same operators and an
exact (LU) solve -- the caller loops of EXAMPLES/COMPLEX/zndrv3.f (mode 2) and
zndrv4.f (mode 3), plus a complex rho with a complex shift
(tests/golden/make_golden.py zmode_fixtures, tests/modes.py ZCaller).

Checks: info, nconv, restart cycles iparam(3), OP*x / B*x counts iparam(9) /
iparam(10) equal to the reference's; every eigenvalue within 1e-9 (relative to
the largest) of the reference's; generalized residuals ||A z - lambda M z|| /
(||A||_1 ||z||) <= 1e-8.  The device solves run to rtol 1e-13 (the
reference's solve is a direct LU)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import modes  # noqa: E402

pytestmark = pytest.mark.gpu


def _zdev(pkg, S):
    S = S.tocsr()
    S.sort_indices()
    return pkg.ZCSR.from_arrays(S.indptr, S.indices, S.data)


@pytest.mark.parametrize("name,method", [("z5_zgen", "bicgstab"), ("z6_zgen_si", "bicgstab"),
                                         ("z7_zgen_si_complex", "bicgstab"), ("z5_zgen", "tridiag"),
                                         ("z6_zgen_si", "tridiag"), ("z7_zgen_si_complex", "tridiag")])
def test_znaupd_generalized_on_device(pkg, golden, name, method):
    """method "tridiag": the direct solve of the tridiagonal C (M in mode 2,
    A - sigma M in mode 3), as zndrv3/zndrv4.f factor it with zgttrf."""
    g = golden(name)
    mode, n, sigma, rho = int(g["mode"]), int(g["n"]), complex(g["sigma"]), complex(g["rho"])
    A, Mm = modes.zconvdiff1d(n, rho)
    G = pkg.ZGen(_zdev(pkg, A), _zdev(pkg, Mm), mode, sigma, rtol=1e-13, maxit=50 * n,
                 method=method)
    s = pkg.ZRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), bmat="G",
                 mode=mode, mxiter=300, v0=g["v0"])
    assert s.aupd_gen(G) == 99
    st = G.stats()
    assert st["fails"] == 0 and st["solves"] > 0, st
    assert (st["iters"] == 0) == (method == "tridiag"), st
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[4]) == int(g["iparam"][4])
    assert int(s.iparam[2]) == int(g["iparam"][2]), (int(s.iparam[2]), int(g["iparam"][2]))
    assert (int(s.iparam[8]), int(s.iparam[9])) == (int(g["iparam"][8]), int(g["iparam"][9]))
    d, z, nconv = s.eupd(sigma=sigma)
    ref = g["d"]
    for x in ref:
        assert np.abs(d - x).min() <= 1e-9 * np.abs(ref).max(), (x, d)
    anorm = abs(A).sum(axis=0).max()
    for k in range(nconv):
        r = A @ z[:, k] - d[k] * (Mm @ z[:, k])
        assert np.linalg.norm(r) / (anorm * np.linalg.norm(z[:, k])) <= 1e-8


def test_zgen_rejects_mismatch(pkg):
    """The operator pair fixes bmat, mode and n: a solve started otherwise
    returns info = -11 (znaupd's mode / bmat code, SRC/znaupd.f:500); a pair
    for a mode other than 2 or 3, or of matrices of different sizes, is
    refused at creation."""
    A, Mm = modes.zconvdiff1d(50, 10.0)
    G = pkg.ZGen(_zdev(pkg, A), _zdev(pkg, Mm), 3, 1.0)
    for bmat, mode in (("G", 2), ("I", 3)):
        s = pkg.ZRci(50, 4, 12, "LM", 1e-10, bmat=bmat, mode=mode, v0=np.ones(50))
        assert s.aupd_gen(G) == 99
        assert int(s.info[0]) == -11, (bmat, mode, int(s.info[0]))
    with pytest.raises(RuntimeError):
        pkg.ZGen(_zdev(pkg, A), _zdev(pkg, Mm), 1, 0j)
    with pytest.raises(RuntimeError):
        pkg.ZGen(_zdev(pkg, A), _zdev(pkg, modes.zconvdiff1d(60, 10.0)[1]), 3, 0j)


@pytest.mark.parametrize("name", ["z5_zgen", "z6_zgen_si", "z7_zgen_si_complex"])
def test_znaupd_generalized_rci(pkg, golden, name):
    """The same fixtures through the reverse-communication loop with the
    reference's own caller (exact LU on the host, tests/modes.py ZCaller): the
    engine's bmat = 'G' path, independent of the device solve -- the
    reference's cycles and OP*x / B*x counts, eigenvalues to 1e-10."""
    g = golden(name)
    mode, n, sigma, rho = int(g["mode"]), int(g["n"]), complex(g["sigma"]), complex(g["rho"])
    c = modes.ZCaller(mode, n, sigma, rho)
    s = pkg.ZRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), bmat="G",
                 mode=mode, mxiter=300, v0=g["v0"])
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            bx = s.slice(2).copy() if ido == 1 else None
            s.slice(1)[:] = c.op(s.slice(0).copy(), ido, bx)
        elif ido == 2:
            s.slice(1)[:] = c.bop(s.slice(0).copy())
        else:
            break
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[2]) == int(g["iparam"][2])
    assert (int(s.iparam[8]), int(s.iparam[9])) == (int(g["iparam"][8]), int(g["iparam"][9]))
    d, _, _ = s.eupd(sigma=sigma)
    np.testing.assert_allclose(np.sort_complex(d), np.sort_complex(g["d"]), rtol=1e-10)
