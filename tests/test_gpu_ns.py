"""GPU parity of the nonsymmetric Arnoldi engine (dnaupd family) against the
reference's golden outputs (tests/golden/n*.npz from oracle/_ref's dnaupd_/
dneupd_ on the same operators and start vectors).

Tolerances:
  * wanted Ritz values |λ - λ_ref| <= max(1e-10, 10*tol) * max|λ_ref| (as sets);
  * restart-cycle counts iparam(3) equal at moderate tol; at tol = eps (n1) and
    on the slowly converging clustered cases (n4, n6: ~450 cycles of a spectrum
    with many equal real parts) the count is rounding-driven, so ±25% there.
"""
import numpy as np
import pytest

from oracle import matrices as M

pytestmark = pytest.mark.gpu

FIXTURES = ["n1_dnsimp", "n2_dnsimp_tol", "n3_convdiff_lm", "n4_convdiff_lr", "n5_convdiff_li",
            "n6_convdiff_sr", "n7_convdiff_real", "n8_convdiff_capped"]
SLOW = {"n1_dnsimp": 0.25, "n4_convdiff_lr": 0.25, "n6_convdiff_sr": 0.25}


def _mat(spec):
    assert str(spec[0]) == "convdiff2d"
    return M.convdiff2d(int(spec[1]), float(spec[2]))


def _check(g, s, name):
    info, iters, nconv = int(s.info[0]), int(s.iparam[2]), int(s.iparam[4])
    ref_iters = int(g["iparam"][2])
    assert info == int(g["info"]), (info, int(g["info"]))
    slack = SLOW.get(name, 0.0)
    assert abs(iters - ref_iters) <= slack * ref_iters, (iters, ref_iters)
    if slack == 0.0:
        assert nconv == int(g["iparam"][4])
    if info == 1:  # capped: same cycles, Ritz estimates close
        return
    lam = s.ritz[:nconv]
    ref = g["ritzr"][:nconv] + 1j * g["ritzi"][:nconv]
    scale = np.abs(ref).max()
    tol = max(1e-10, 10 * float(g["tol"])) * scale
    for z in ref:  # every reference Ritz value is matched by one of ours
        assert np.abs(lam - z).min() <= tol, (z, lam)


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
