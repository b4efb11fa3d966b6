"""GPU parity of the nonsymmetric Arnoldi engine (dnaupd family) against the
reference's golden outputs (tests/golden/n*.npz from oracle/_ref's dnaupd_/
dneupd_ on the same operators and start vectors).

Ritz-value criteria (adapted to non-normal operators):
  * backward error: every Ritz value λ we return lies in the tol-pseudospectrum,
    σ_min(A - λI) <= 100·max(tol, eps)·||A||_1 (dense SVD, n <= 2500), and the
    same holds for the reference's values -- conv-diff with strong convection is
    far from normal, so individual eigenvalues are ill-conditioned (n3: the
    reference's own Ritz value and its dneupd eigenvalue differ by 1.3e-4) and
    no implementation pins them to 1e-10;
  * selection: the sorted `which` keys (|λ| for LM/SM, Re for LR/SR, |Im| for
    LI/SI) agree with the reference's to 1e-6 relative -- with ties in the key
    (n4/n6: all wanted values share one real part) WHICH tied values are
    returned is rounding-determined in the reference too;
  * restart-cycle counts iparam(3) equal at moderate tol; at tol = eps (n1) ±25%;
    the slowly converging tied cases (n4, n6: 400-500 cycles) only need info = 0
    and nconv = nev.
"""
import numpy as np
import pytest

from oracle import matrices as M

pytestmark = pytest.mark.gpu

FIXTURES = ["n1_dnsimp", "n2_dnsimp_tol", "n3_convdiff_lm", "n4_convdiff_lr", "n5_convdiff_li",
            "n6_convdiff_sr", "n7_convdiff_real", "n8_convdiff_capped"]
SLOW = {"n1_dnsimp": 0.25, "n4_convdiff_lr": None, "n6_convdiff_sr": None}


def _mat(spec):
    assert str(spec[0]) == "convdiff2d"
    return M.convdiff2d(int(spec[1]), float(spec[2]))


def _check(g, s, name):
    info, iters, nconv = int(s.info[0]), int(s.iparam[2]), int(s.iparam[4])
    ref_iters = int(g["iparam"][2])
    assert info == int(g["info"]), (info, int(g["info"]))
    slack = SLOW.get(name, 0.0)
    if slack is None:
        assert nconv >= int(g["nev"])
    else:
        assert abs(iters - ref_iters) <= slack * ref_iters, (iters, ref_iters)
    if slack == 0.0:
        assert nconv == int(g["iparam"][4])
    if info == 1:  # capped: same cycles, Ritz estimates close
        return
    lam = s.ritz[:nconv]
    ref = g["ritzr"][:nconv] + 1j * g["ritzi"][:nconv]
    _ritz_ok(_mat(g["spec"]), lam, ref, str(g["which"]), float(g["tol"]))


KEYS = {"LM": np.abs, "SM": np.abs, "LR": np.real, "SR": np.real,
        "LI": lambda z: np.abs(np.imag(z)), "SI": lambda z: np.abs(np.imag(z))}


def _ritz_ok(mat, lam, ref, which, tol):
    A = M.to_scipy(*mat)
    n = A.shape[0]
    nm = min(len(lam), len(ref))
    key = KEYS[which]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(np.sort(key(lam))[-nm:], np.sort(key(ref))[-nm:], rtol=0,
                               atol=1e-6 * scale)
    if n <= 2500:
        D = A.toarray()
        anorm = np.abs(D).sum(axis=0).max()
        bound = 100 * max(tol, np.finfo(float).eps) * anorm
        for z in list(lam) + list(ref):
            smin = np.linalg.svd(D - z * np.eye(n), compute_uv=False)[-1]
            assert smin <= bound, (z, smin, bound)
    else:  # well-conditioned (real) spectrum: direct comparison
        for z in ref[:nm]:
            assert np.abs(lam - z).min() <= max(1e-10, 10 * tol) * scale, (z, lam)


@pytest.mark.parametrize("name", FIXTURES)
def test_dnaupd_rci_host_op(pkg, golden, name):
    """Reference RCI contract: the caller applies OP (scipy CSR) on host arrays."""
    g = golden(name)
    rp, col, val = _mat(g["spec"])
    A = M.to_scipy(rp, col, val)
    n = A.shape[0]
    s = pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]),
                  mxiter=int(g["mxiter"]), v0=g["v0"])
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        elif ido == 99:
            break
        else:
            raise AssertionError(ido)
    _check(g, s, name)


@pytest.mark.parametrize("name", FIXTURES)
def test_dnaupd_csr_free_run(pkg, golden, name):
    """Whole Arnoldi loop on the GPU, OP = device CSR from the device generator."""
    g = golden(name)
    spec = g["spec"]
    Ad = pkg.CSR.convdiff2d(int(spec[1]), float(spec[2]))
    n = int(spec[1]) ** 2
    s = pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]),
                  mxiter=int(g["mxiter"]), v0=g["v0"], device=True)
    assert s.aupd_csr(Ad) == 99
    _check(g, s, name)


def test_convdiff_generator_bitwise(pkg):
    for m, rho in [(10, 100.0), (37, 3.5)]:
        rp, col, val = M.convdiff2d(m, rho)
        drp, dcol, dval = pkg.CSR.convdiff2d(m, rho).download()
        assert np.array_equal(rp, drp) and np.array_equal(col, dcol) and np.array_equal(val, dval)


def _eigvecs(z, dr, di):
    """Columns of dneupd's Z -> complex eigenvectors (pair j, j+1 = re, im)."""
    out, j = [], 0
    while j < len(dr):
        if di[j] == 0.0:
            out.append(z[:, j].astype(complex))
            j += 1
        else:
            x = z[:, j] + 1j * z[:, j + 1]
            out += [x, x.conj()]
            j += 2
    return out[:len(dr)]


def _max_resid(A, z, dr, di):
    anorm = abs(A).sum(axis=0).max()
    r = 0.0
    for x, lam in zip(_eigvecs(z, dr, di), dr + 1j * di):
        r = max(r, np.linalg.norm(A @ x - lam * x) / (anorm * np.linalg.norm(x)))
    return r


@pytest.mark.parametrize("name", ["n1_dnsimp", "n2_dnsimp_tol", "n3_convdiff_lm", "n5_convdiff_li",
                                  "n7_convdiff_real"])
@pytest.mark.parametrize("device", [False, True])
def test_dneupd_ritz_vectors(pkg, golden, name, device):
    """dneupd (SRC/dneupd.f): eigenvalues equal the reference's dr/di and the
    Ritz vectors' residuals ||Ax - λx|| / (||A||_1 ||x||) are no worse than 10x
    the reference's own (fixtures without reference vectors: 10x tol)."""
    g = golden(name)
    spec = g["spec"]
    rp, col, val = _mat(spec)
    A = M.to_scipy(rp, col, val)
    n = A.shape[0]
    s = pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]), float(g["tol"]),
                  mxiter=int(g["mxiter"]), v0=g["v0"], device=device)
    if device:
        assert s.aupd_csr(pkg.CSR.convdiff2d(int(spec[1]), float(spec[2]))) == 99
    else:
        while s.aupd() in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
    assert s.info[0] == 0
    dr, di, z, nconv = s.eupd()
    assert s.eupd_info == int(g["eupd_info"]) == 0
    assert nconv == len(g["dr"])
    z = (z.numpy() if device else z).reshape(int(g["nev"]) + 1, n)[:nconv].T
    lam, ref = dr + 1j * di, g["dr"] + 1j * g["di"]
    _ritz_ok((rp, col, val), lam, ref, str(g["which"]), float(g["tol"]))
    ours = _max_resid(A, z, dr, di)
    theirs = _max_resid(A, g["z"], g["dr"], g["di"]) if "z" in g else float(g["tol"])
    assert ours <= max(10 * theirs, 1e-12), (ours, theirs)
    if name == "n2_dnsimp_tol":  # well separated: vectors equal the reference's up to phase
        for x, lam_x in zip(_eigvecs(z, dr, di), lam):
            k = int(np.argmin(np.abs(ref - lam_x)))
            xr = _eigvecs(g["z"], g["dr"], g["di"])[k]
            c = np.vdot(xr, x) / np.vdot(xr, xr)
            assert abs(abs(c) - 1) < 1e-8
            np.testing.assert_allclose(x, c * xr, atol=1e-8)
