"""GPU: device errors reach the caller.

The engine keeps the first failed HIP call of a solve (a copy, an enqueue, or a
kernel fault surfacing at a stream sync) as a sticky per-solve record and ends
the solve with info = -9999 at its next return, as the reference's drivers end
on a failed step (SRC/dsaup2.f:371-375: info = -9999 from dsaitr).  The hook
arpack_hip_fault_inject(k) makes the k-th checked call report
hipErrorInvalidValue; these tests sweep it over the RCI and free-running
dsaupd/dnaupd paths, dseupd, znaupd and the CSR plan builders, and check that
every injection ends in -9999 / -2 (never a hang, a crash or a silently wrong
answer) and that the next, unarmed solve is exact again.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import matrices as M

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _disarm(pkg):
    pkg.fault_inject(0)
    yield
    pkg.fault_inject(0)


def _lap(m):
    return M.to_scipy(*M.laplace2d(m))


def _rci_solve(pkg, A, n, arm=0, cls="SymRci", which="LM"):
    s = getattr(pkg, cls)(n, 6, 20, which, 1e-10, mxiter=300, v0=np.linspace(-1, 1, n))
    ido = s.aupd()
    if arm:
        pkg.fault_inject(arm)
    while ido != 99:
        assert ido in (-1, 1), ido
        s.slice(1)[:] = A @ s.slice(0)
        ido = s.aupd()
    pkg.fault_inject(0)
    return s


@pytest.mark.timeout(300)
@pytest.mark.parametrize("cls", ["SymRci", "NsRci"])
def test_rci_injection_sweep_ends_in_9999(pkg, cls):
    m = 30
    A = _lap(m)
    n = m * m
    good = _rci_solve(pkg, A, n, cls=cls)
    assert int(good.info[0]) == 0
    ref = (int(good.iparam[2]), int(good.iparam[8]))
    hit = 0
    for k in list(range(1, 30)) + [37, 61, 97, 151, 233, 401]:
        s = _rci_solve(pkg, A, n, arm=k, cls=cls)
        info = int(s.info[0])
        if info == 0:  # the k-th call came after the solve ended
            assert (int(s.iparam[2]), int(s.iparam[8])) == ref
        else:
            assert info == -9999, (k, info)
            hit += 1
    assert hit >= 25
    again = _rci_solve(pkg, A, n, cls=cls)
    assert int(again.info[0]) == 0 and (int(again.iparam[2]), int(again.iparam[8])) == ref


@pytest.mark.timeout(300)
@pytest.mark.parametrize("cls", ["SymRci", "NsRci"])
def test_free_running_injection_ends_in_9999(pkg, cls):
    m = 40
    n = m * m
    A = pkg.CSR.laplace2d(m)
    v0 = np.linspace(-1, 1, n)

    def solve(arm):
        s = getattr(pkg, cls)(n, 6, 20, "LM", 1e-10, mxiter=300, v0=v0)
        if arm:
            pkg.fault_inject(arm)
        s.aupd_csr(A)
        pkg.fault_inject(0)
        return s
    good = solve(0)
    assert int(good.info[0]) == 0
    for k in (1, 2, 3, 5, 8, 13, 21, 34, 55):
        s = solve(k)
        assert int(s.ido[0]) == 99
        assert int(s.info[0]) == -9999, (k, int(s.info[0]))
    again = solve(0)
    assert int(again.info[0]) == 0
    assert int(again.iparam[2]) == int(good.iparam[2])


@pytest.mark.timeout(120)
def test_seupd_injection(pkg):
    m = 30
    A = _lap(m)
    s = _rci_solve(pkg, A, m * m)
    assert int(s.info[0]) == 0
    pkg.fault_inject(2)
    with pytest.raises(pkg.ArpackError) as e:
        s.eupd(rvec=True)
    assert e.value.info == -9999


@pytest.mark.timeout(120)
def test_znaupd_injection(pkg):
    n = 800
    A = M.to_scipy(*M.zrandom(n, 10, 3, 10.0))
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)

    def solve(arm):
        s = pkg.ZRci(n, 6, 20, "LM", 1e-10, mxiter=300, v0=v0)
        ido = s.aupd()
        if arm:
            pkg.fault_inject(arm)
        while ido != 99:
            assert ido in (-1, 1), ido
            s.slice(1)[:] = A @ s.slice(0)
            ido = s.aupd()
        pkg.fault_inject(0)
        return s
    good = solve(0)
    assert int(good.info[0]) == 0
    for k in (1, 4, 9, 16, 25, 49):
        assert int(solve(k).info[0]) == -9999, k
    assert int(solve(0).iparam[2]) == int(good.iparam[2])


@pytest.mark.timeout(120)
def test_csr_create_plan_failure_returns_minus2(pkg):
    rp, col, val = M.laplace2d(50)
    L = pkg.lib()
    for k in (1, 2, 3, 4, 6, 9):
        h = C.c_void_p()
        pkg.fault_inject(k)
        rc = L.arpack_hip_csr_create(C.byref(h), len(rp) - 1, len(col), rp.ctypes.data,
                                     col.ctypes.data, val.ctypes.data)
        pkg.fault_inject(0)
        if rc == 0:  # k past the plan builders' calls
            L.arpack_hip_csr_destroy(h)
            continue
        assert rc == -2, (k, rc)
        assert not h.value  # nothing handed out
    A = pkg.CSR.from_arrays(rp, col, val)  # the next create is whole again
    x = np.linspace(-1, 1, len(rp) - 1)
    xd = pkg.DeviceBuffer.from_numpy(x)
    yd = pkg.DeviceBuffer(len(x))
    A.matvec_device(xd, yd)
    np.testing.assert_array_equal(yd.numpy(), M.to_scipy(rp, col, val) @ x)
