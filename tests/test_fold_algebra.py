"""CPU: the algebra of the folded Lanczos / Arnoldi step (DESIGN.md §2,
arpack-ng_amd/csrc/fold.hip), restated in numpy next to the reference's step
order (SRC/dsaitr.f:569-583 CGS, :680-692 DGKS; SRC/dnaitr.f the same with a
full Hessenberg column).

Reference order per step j:  w = A v_j;  h = V' w;  r = w - V h;  s = V' r;
r' = r - V s;  beta = |r'|;  v_{j+1} = r' / beta  (DGKS taken every step here).
Folded order: the SpMV runs on r (before its sweep), and the next step rebuilds
A r' = A r - V (H s) - s_j r'  from the Arnoldi relation A V = V H + r' e'.
The two must produce the same H (to rounding) and an orthonormal basis."""
import numpy as np
import pytest


def _reference(A, v0, m, sym):
    n = A.shape[0]
    V = np.zeros((n, m + 1))
    H = np.zeros((m + 1, m))
    V[:, 0] = v0 / np.linalg.norm(v0)
    for j in range(m):
        w = A @ V[:, j]
        h = V[:, :j + 1].T @ w
        r = w - V[:, :j + 1] @ h
        s = V[:, :j + 1].T @ r
        r = r - V[:, :j + 1] @ s
        H[:j + 1, j] = h + s
        H[j + 1, j] = np.linalg.norm(r)
        V[:, j + 1] = r / H[j + 1, j]
    if sym:  # dsaitr keeps only the tridiagonal part (h(j,1), h(j,2) + s_j)
        H = np.triu(np.tril(H, 1), -1)
    return V, H


def _folded(A, v0, m, sym):
    """Step 1 as the reference; steps 2..m: the SpMV on the pre-sweep r."""
    n = A.shape[0]
    V = np.zeros((n, m + 1))
    H = np.zeros((m + 1, m))
    V[:, 0] = v0 / np.linalg.norm(v0)
    y = A @ V[:, 0]
    r_pre = s_prev = None
    for j in range(m):
        J = j + 1  # formed columns after this step
        if j == 0:
            w = y
        else:
            # fold: r' = r - V s (step j-1's sweep), w = A r' / beta from y = A r
            Vp = V[:, :j]
            rp = r_pre - Vp @ s_prev
            T = H[:j, :j]                      # (tridiagonal for Lanczos)
            t = T @ s_prev
            beta = np.linalg.norm(rp)
            H[j, j - 1] = beta
            V[:, j] = rp / beta
            w = (y - Vp @ t - s_prev[-1] * rp) / beta
        h = V[:, :J].T @ w
        r = w - V[:, :J] @ h
        s = V[:, :J].T @ r
        H[:J, j] = h + s
        if sym and J > 2:
            H[:J - 2, j] = 0.0  # the tridiagonal records only
        if j == m - 1:  # the last step takes its sweep as a pass of its own
            rp = r - V[:, :J] @ s
            H[J, j] = np.linalg.norm(rp)
            V[:, J] = rp / H[J, j]
            break
        y = A @ r  # the SpMV of the next step, on r before its sweep
        r_pre, s_prev = r, s
    return V, H


@pytest.mark.parametrize("sym", [True, False])
def test_folded_step_equals_reference_order(sym):
    rng = np.random.default_rng(11)
    n, m = 600, 40
    B = rng.standard_normal((n, n)) * (rng.random((n, n)) < 0.02)
    A = (B + B.T) / 2 + np.diag(np.linspace(0, 30, n)) if sym else B + np.diag(np.linspace(0, 30, n))
    v0 = rng.uniform(-1, 1, n)
    V1, H1 = _reference(A, v0, m, sym)
    V2, H2 = _folded(A, v0, m, sym)
    scale = np.abs(H1).max()
    assert np.abs(H1 - H2).max() <= 1e-13 * scale, np.abs(H1 - H2).max() / scale  # measured ~5e-16
    for V in (V1, V2):
        assert np.abs(V.T @ V - np.eye(m + 1)).max() < 1e-12
    # the Arnoldi relation A V_m = V_{m+1} H holds for the folded basis too
    res = A @ V2[:, :m] - V2 @ H2
    tol = 1e-9 if sym else 1e-12  # (Lanczos drops the off-tridiagonal O(eps) entries)
    assert np.abs(res).max() <= tol * scale
