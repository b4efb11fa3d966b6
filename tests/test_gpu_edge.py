"""GPU edge cases against the reference run in-process (oracle/_ref), same
operator and start vector:

* rank-deficient operators: the Krylov space is exhausted after rank+1 steps, so
  the residual collapses to rounding noise -- the DGKS give-up / zero residual
  (SRC/dsaitr.f:753-781) and the invariant-subspace restart through dgetv0
  (SRC/dsaitr.f:378-436, SRC/dgetv0.f:326-397) paths (on rank3_lm the
  reference takes 5 such restarts and 12 refinement steps in one cycle);
* the smallest legal problems (n = 2, 3; ncv = n: the full Krylov space);
* one shift per cycle (np = ncv - nev = 1);
* which = 'BE' with an odd nev (SRC/dsgets.f:151-176 splits the extra one to the
  high end).

Ritz values: |d - d_ref| <= 1e-9 * max(1, |d_ref|max).  Restart cycles equal,
except where the path is decided by rounding noise (rank-deficient operators:
whether a noise-sized residual passes the 0.717 test depends on the last ulp of
the sums), which get two cycles of slack.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import matrices as M
from oracle import ref

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not ref.available(), reason="oracle/_ref")]


def _sym_cases():
    rng = np.random.default_rng(11)
    B = rng.integers(-8, 9, size=(12, 12)) / 8.0
    dense12 = sp.csr_matrix(B + B.T)
    rank3 = sp.diags(np.r_[1.0, 2.0, 3.0, np.zeros(97)]).tocsr()
    return {
        # name: (A, nev, ncv, which, tol, mxiter, noisy)
        "rank3_lm": (rank3, 2, 8, "LM", 1e-10, 300, True),
        "full_krylov_n12": (dense12, 4, 12, "LA", 0.0, 300, False),
        "tiny_n3": (sp.diags([1.0, 2.0, 3.0]).tocsr(), 1, 3, "LM", 0.0, 300, False),
        "tiny_n2": (sp.csr_matrix(np.array([[2.0, 1.0], [1.0, 3.0]])), 1, 2, "LA", 0.0, 300,
                    False),
        "np1_anderson": (M.to_scipy(*M.anderson(20, 2, 4.0, 7)), 9, 10, "LA", 1e-8, 3000, False),
        "be_odd_anderson": (M.to_scipy(*M.anderson(20, 2, 4.0, 7)), 5, 16, "BE", 1e-9, 3000,
                            False),
    }


SYM = _sym_cases()


def _close(d, dref):
    d, dref = np.sort(np.asarray(d)), np.sort(np.asarray(dref))
    assert len(d) == len(dref)
    scale = max(1.0, np.abs(dref).max()) if len(dref) else 1.0
    assert np.all(np.abs(d - dref) <= 1e-9 * scale), (d, dref)


@pytest.mark.parametrize("device", [False, True])
@pytest.mark.parametrize("name", list(SYM))
def test_dsaupd_edge(pkg, name, device):
    A, nev, ncv, which, tol, mx, noisy = SYM[name]
    n = A.shape[0]
    v0 = M.dlarnv_uniform(n)[0]
    want = ref.dsaupd_solve(lambda x, *_: A @ x, n, nev, ncv, which, tol, v0=v0, mxiter=mx)
    if device:  # whole loop on the GPU, OP = device CSR
        op = pkg.CSR.from_arrays(A.indptr.astype(np.int64), A.indices, A.data)
    else:       # reference RCI contract, caller's OP on host arrays
        op = lambda x: A @ x  # noqa: E731
    d, z, res = pkg.eigsh(op, n, nev, ncv, which, tol, v0=v0, mxiter=mx, device=device)
    assert res["info"] == want["info"]
    assert res["nconv"] == want["nconv"]
    slack = 2 if noisy else 0
    assert abs(res["iters"] - int(want["iparam"][2])) <= slack, (res, want["iparam"])
    _close(d, want["d"])
    # Ritz vectors: A z = d z
    r = np.linalg.norm(A @ z - z * d, axis=0)
    assert np.all(r <= 1e-8 * max(1.0, np.abs(d).max())), r


def _dense_ns14():
    # well-conditioned nonsymmetric 14 x 14 (eigenvector condition ~5.6; three
    # complex pairs).  A tiny convection-diffusion block is NOT used here: its
    # clustered eigenvalues are so ill-conditioned that the reference's own Ritz
    # values sit 1e-2 away from the true ones, i.e. any rounding difference
    # reorders the wanted set.
    rng = np.random.default_rng(5)
    return sp.csr_matrix(rng.integers(-8, 9, size=(14, 14)) / 8.0 + np.diag(np.arange(14.0)))


NS = {
    "full_krylov_n14_lm": (_dense_ns14(), 4, 14, "LM", 0.0, False),
    "full_krylov_n14_lr": (_dense_ns14(), 3, 14, "LR", 0.0, False),
    "rank3_lm": (sp.diags(np.r_[1.0, 2.0, 3.0, np.zeros(57)]).tocsr(), 2, 8, "LM", 1e-10, True),
    "np2_convdiff": (M.to_scipy(*M.convdiff2d(10, 10.0)), 6, 8, "LR", 1e-8, False),
}


@pytest.mark.parametrize("name", list(NS))
def test_dnaupd_edge(pkg, name):
    A, nev, ncv, which, tol, noisy = NS[name]
    n = A.shape[0]
    v0 = M.dlarnv_uniform(n)[0]
    want = ref.dnaupd_solve(lambda x, *_: A @ x, n, nev, ncv, which, tol, v0=v0, mxiter=3000,
                            rvec=False)
    s = pkg.NsRci(n, nev, ncv, which, tol, mxiter=3000, v0=v0)
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        elif ido == 99:
            break
        else:
            raise AssertionError(ido)
    assert int(s.info[0]) == want["info"]
    slack = 2 if noisy else 0
    assert abs(int(s.iparam[2]) - int(want["iparam"][2])) <= slack
    dr, di, _, nconv = s.eupd(rvec=False)
    assert nconv == want["nconv"]
    got = np.sort_complex(dr[:nconv] + 1j * di[:nconv])
    exp = np.sort_complex(want["dr"] + 1j * want["di"])
    assert np.all(np.abs(got - exp) <= 1e-9 * max(1.0, np.abs(exp).max())), (got, exp)


def test_znaupd_full_krylov(pkg):
    """znaupd with ncv = n (the complex diagonal operator of TESTS/icb_arpack_c.c, n = 12)."""
    n, nev, ncv = 12, 3, 12
    dg = np.array([complex(i + 1, i + 1) for i in range(n)])
    A = sp.diags(dg).tocsr()
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)
    want = ref.znaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LM", 0.0, v0=v0, rvec=False)
    s = pkg.ZRci(n, nev, ncv, "LM", 0.0, v0=v0)
    while True:
        ido = s.aupd()
        if ido in (-1, 1):
            s.slice(1)[:] = A @ s.slice(0)
        elif ido == 99:
            break
        else:
            raise AssertionError(ido)
    assert int(s.info[0]) == want["info"]
    assert int(s.iparam[2]) == int(want["iparam"][2])
    d, _, nconv = s.eupd(rvec=False)
    assert nconv == want["nconv"]
    got, exp = np.sort_complex(d[:nconv]), np.sort_complex(want["d"])
    assert np.all(np.abs(got - exp) <= 1e-9 * max(1.0, np.abs(exp).max())), (got, exp)


def test_chained_steps_range_guard(pkg):
    """Chained free-running Lanczos steps run OP on the raw residual r instead
    of v = r / rnorm; a residual norm outside [1e-150, 1e150] parks the step
    (abort = 3) and the host redoes it with v formed first.  An operator scaled
    by 2^500 (~3e150) puts the early residual norms above the range (later ones,
    shrinking with convergence, fall back inside it), so both paths alternate.
    Power-of-two scaling is exact in every operation of the reference, so its
    results for the scaled operator are its unscaled ones times 2^500: Ritz
    values, restart cycles and OP*x counts must match.  (Norms here are
    sqrt(sum x^2), not dnrm2's scaled sum -- DESIGN.md §2 -- so a scale that
    pushes sum x^2 past the double range, 2^600 or 2^-510, is outside what
    either path supports; the guard keeps the raw path inside it.)"""
    e = 500
    A = M.to_scipy(*M.anderson(20, 2, 4.0, 7))
    As = (A * 2.0 ** e).tocsr()
    n, nev, ncv = A.shape[0], 6, 20
    v0 = M.dlarnv_uniform(n)[0]
    want = ref.dsaupd_solve(lambda x, *_: As @ x, n, nev, ncv, "LA", 1e-9, v0=v0, mxiter=3000)
    base = ref.dsaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LA", 1e-9, v0=v0, mxiter=3000)
    assert int(want["iparam"][2]) == int(base["iparam"][2])  # the scaling is exact
    op = pkg.CSR.from_arrays(As.indptr.astype(np.int64), As.indices, As.data)
    d, z, res = pkg.eigsh(op, n, nev, ncv, "LA", 1e-9, v0=v0, mxiter=3000, device=False)
    assert res["info"] == want["info"] == 0
    assert res["iters"] == int(want["iparam"][2])
    assert res["nopx"] == int(want["iparam"][8])
    d0 = d * 2.0 ** -e
    _close(d0, np.asarray(want["d"]) * 2.0 ** -e)
    r = np.linalg.norm(A @ z - z * d0, axis=0)
    assert np.all(r <= 1e-8 * max(1.0, np.abs(d0).max())), r
