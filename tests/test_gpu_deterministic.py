"""GPU: deterministic mode (arpack_hip_set_deterministic).

The upper-triangle symmetric SpMV and the complex row-tile SpMV accumulate in
LDS with atomics in wave-schedule order, so a solve through them reproduces its
Ritz values to ~1e-15 but not bit for bit.  Deterministic mode keeps only
fixed-order forms (full-storage SELL, bitwise SciPy's csr_matvec; the complex
column-split kernel): repeated solves must then agree BITWISE, and the
declared-symmetric call reports that it kept full storage (rc = 1).
"""
import numpy as np
import pytest

from oracle import matrices as M

pytestmark = pytest.mark.gpu


@pytest.fixture
def det(pkg):
    pkg.set_deterministic(True)
    yield
    pkg.set_deterministic(False)


def test_symmetric_declaration_keeps_full_storage(pkg, det):
    A = pkg.CSR.banded_sym(200_000, 1234, 4096, 25)
    A.set_symmetric(True)
    assert A.last_rc == 1 and not A.symmetric
    n = A.n
    v0 = M.dlarnv_uniform(n)[0]
    runs = []
    for _ in range(3):
        s = pkg.SymRci(n, 10, 30, "LA", 1e-8, mxiter=300, device=True, v0=v0)
        assert s.aupd_csr(A) == 99 and int(s.info[0]) == 0
        d, _, nconv = s.eupd(rvec=False)
        runs.append((int(s.iparam[2]), int(s.iparam[8]), d[:nconv].copy()))
    for r in runs[1:]:
        assert r[:2] == runs[0][:2]
        np.testing.assert_array_equal(r[2], runs[0][2])  # bitwise


def test_deterministic_off_restores_symmetric(pkg):
    pkg.set_deterministic(False)
    A = pkg.CSR.banded_sym(200_000, 1234, 4096, 25)
    A.set_symmetric(True)
    assert A.last_rc == 0 and A.symmetric


def test_complex_operator_bitwise_repeatable(pkg, det):
    n = 100_000
    Z = pkg.ZCSR.random(n, 100, 5, 100.0)
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)
    x = (np.arange(n) % 7 - 3.0) + 1j * (np.arange(n) % 5 - 2.0)
    y0 = Z.matvec(x)
    for _ in range(3):
        np.testing.assert_array_equal(Z.matvec(x), y0)
    runs = []
    for _ in range(2):
        s = pkg.ZRci(n, 6, 20, "LM", 1e-8, mxiter=6, v0=v0)  # capped: Ritz values in workl
        s.aupd_zcsr(Z)
        runs.append((int(s.iparam[2]), np.array(s.ritz)))
    assert runs[0][0] == runs[1][0]
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
