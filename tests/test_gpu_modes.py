"""GPU parity of the spectral-transformation modes (§8 f2): the engine driven
through the RCI contract by the same caller operators (tests/modes.py) the
reference was driven with to make tests/golden/m*.npz.

  dsaupd modes 3 (bmat I and G), 2, 4 (buckling), 5 (Cayley) with dseupd's
  back-transformations; dnaupd modes 3 (bmat I, G) and 2 with dneupd.
Checks: info, nconv, restart cycles iparam(3), OP*x / B*x counts equal to the
reference; eigenvalues within 1e-9 relative; generalized residuals
||A z - λ M z|| / (||A||_1 ||z||) <= 1e-8 (buckling: K = A, KG = M)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import modes  # noqa: E402

pytestmark = pytest.mark.gpu

SYM = ["m2_sym_std_si", "m3_sym_gen", "m4_sym_gen_si", "m5_sym_buckling", "m6_sym_cayley"]
NS = ["m7_ns_std_si", "m8_ns_gen", "m9_ns_gen_si"]


def _caller(g, name):
    kind, mode, n, sigma = str(g["kind"]), int(g["mode"]), int(g["n"]), float(g["sigma"])
    if "_std_" in name:  # bmat = 'I' shift-invert (dsdrv2 / dndrv2)
        return modes.StdShiftInvert(kind, n, sigma)
    return modes.Caller(kind, mode, n, sigma)


def _drive(s, c, n):
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            bx = s.slice(2).copy() if (c.mode >= 3 and ido == 1) else None
            y = c.op(s.slice(0).copy(), ido, bx)
            s.slice(1)[:] = y
            if c.mode == 2:
                s.slice(0)[:] = c.ax
        elif ido == 2:
            s.slice(1)[:] = c.bop(s.slice(0).copy())
        elif ido == 99:
            return
        else:
            raise AssertionError(ido)


def _stats(pkg):
    st = pkg.stats()
    return st["nopx"], st["nbx"]


@pytest.mark.parametrize("name", SYM)
def test_dsaupd_modes(pkg, golden, name):
    g = golden(name)
    c = _caller(g, name)
    n = int(g["n"])
    s = pkg.SymRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), bmat=c.bmat,
                   mode=c.mode, mxiter=300, v0=g["v0"])
    _drive(s, c, n)
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[4]) == int(g["iparam"][4])
    assert int(s.iparam[2]) == int(g["iparam"][2])
    assert (int(s.iparam[8]), int(s.iparam[9])) == (int(g["iparam"][8]), int(g["iparam"][9]))
    d, z, nconv = s.eupd(sigma=float(g["sigma"]))
    np.testing.assert_allclose(np.sort(d), np.sort(g["d"]), rtol=1e-9)
    z = z.reshape(int(g["nev"]), n)[:nconv].T
    A = c.A
    Bm = getattr(c, "M", None)
    anorm = abs(A).sum(axis=0).max()
    for k in range(nconv):
        lhs = A @ z[:, k]
        rhs = d[k] * (Bm @ z[:, k] if Bm is not None else z[:, k])
        assert np.linalg.norm(lhs - rhs) / (anorm * np.linalg.norm(z[:, k])) <= 1e-8


@pytest.mark.parametrize("name", NS)
def test_dnaupd_modes(pkg, golden, name):
    g = golden(name)
    c = _caller(g, name)
    n = int(g["n"])
    s = pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), bmat=c.bmat,
                  mode=c.mode, mxiter=300, v0=g["v0"])
    _drive(s, c, n)
    assert int(s.info[0]) == int(g["info"]) == 0
    assert int(s.iparam[4]) == int(g["iparam"][4])
    assert int(s.iparam[2]) == int(g["iparam"][2])
    dr, di, z, nconv = s.eupd(sigmar=float(g["sigma"]))
    lam, ref = dr + 1j * di, g["dr"] + 1j * g["di"]
    for x in ref:
        assert np.abs(lam - x).min() <= 1e-9 * np.abs(ref).max(), (x, lam)
