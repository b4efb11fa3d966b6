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


# Z = V: the reference's drivers pass v for z (TESTS/bug_58_double.f:294,
# EXAMPLES/NONSYM/dndrv2.f), and the reference then leaves the Ritz vectors in
# V(:,1:nconv). The vectors must be the ones a separate Z receives, bit for bit.
@pytest.mark.parametrize("name", ["m2_sym_std_si", "m7_ns_std_si"])
def test_eupd_z_aliases_v(pkg, golden, name):
    g = golden(name)
    n = int(g["n"])
    out = []
    for alias in (False, True):
        c = _caller(g, name)
        cls = pkg.SymRci if name in SYM else pkg.NsRci
        s = cls(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), bmat=c.bmat,
                mode=c.mode, mxiter=300, v0=g["v0"])
        _drive(s, c, n)
        zarg = s.v if alias else None
        if name in SYM:
            d, z, nconv = s.eupd(sigma=float(g["sigma"]), z=zarg)
        else:
            d, _, z, nconv = s.eupd(sigmar=float(g["sigma"]), z=zarg)
        out.append((d.copy(), np.array(z[:nconv * n]).copy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


def test_zneupd_z_aliases_v(pkg, golden):
    import scipy.sparse as sp
    import scipy.sparse.linalg as spl
    from oracle import matrices as M
    g = golden("z3_zrandom_si")
    rp, col, val = M.zrandom(*(int(x) for x in g["spec"][1:4]), float(g["spec"][4]))
    n = len(rp) - 1
    A = sp.csr_matrix((val, col, rp), shape=(n, n))
    lu = spl.splu(A.tocsc())
    out = []
    for alias in (False, True):
        s = pkg.ZRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]), mode=3,
                     mxiter=int(g["mxiter"]), v0=g["v0"])
        while (ido := s.aupd()) in (-1, 1):
            s.slice(1)[:] = lu.solve(s.slice(0).copy())
        assert ido == 99
        d, z, nconv = s.eupd(sigma=complex(g["sigma"]), z=s.v if alias else None)
        out.append((d.copy(), z.copy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
