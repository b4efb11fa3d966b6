"""CPU: the host BiCGStab restatement of the device shift-invert solve
(oracle/krylov.py, the checker of arpack-ng_amd/csrc/zsolve.hip) against a dense
direct solve -- pins the oracle of the mode-3 OP on first principles."""
import numpy as np
import pytest

from oracle.krylov import bicgstab
from oracle import matrices as M


@pytest.mark.parametrize("sigma", [0j, 0.5 + 0.25j, 90.0 - 1.0j])
def test_bicgstab_matches_direct_solve(sigma):
    n = 600
    rp, col, val = M.zrandom(n, 40, 11, 100.0)
    A = M.to_scipy(rp, col, val).toarray()
    rng = np.random.default_rng(3)
    b = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    y, it, rr, ok = bicgstab(lambda x: A @ x, b, sigma, 1e-13)
    assert ok and it > 0 and rr <= 1e-13
    ref = np.linalg.solve(A - sigma * np.eye(n), b)
    assert np.linalg.norm(y - ref) <= 1e-11 * np.linalg.norm(ref)


def test_bicgstab_zero_rhs_and_maxit():
    n = 200
    rp, col, val = M.zrandom(n, 20, 1, 100.0)
    A = M.to_scipy(rp, col, val)
    y, it, rr, ok = bicgstab(lambda x: A @ x, np.zeros(n, complex))
    assert ok and it == 0 and not y.any()
    b = np.ones(n, complex)
    _, it, rr, ok = bicgstab(lambda x: A @ x, b, 0j, 1e-30, maxit=2)
    assert not ok and it == 2
