"""GPU: every device-pointer ABI entry orders itself behind the caller's own GPU
work (the RCI contract, SRC/dsaupd.f:228-234: the arrays
are complete when *aupd / *eupd is called).

The caller's in-flight work is stood in for by arpack_hip_test_delayed_fill: a
kernel on a private non-blocking stream that waits 50-80 ms on the device clock
and only then writes the array.  Each entry is called right after it, and its
results are compared word for word with the same call on a synchronously
written array:
  * dsaupd (ido = 0, info = 1) reading a device resid the caller is still writing;
  * dseupd_c writing a device Z the caller is still overwriting (the bug class
    behind round 4's 8-rank failure: zero Ritz-vector rows);
  * arpack_hip_csr_spmv reading a device x the caller is still writing.
Without the ordering, the engine reads zeros (resid, x) or its Z is overwritten
by the late fill."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, NEV, NCV = 200_000, 6, 20
DELAY_US = 80_000


def _fill(pkg, dst, src, value, count):
    L = pkg.lib()
    L.arpack_hip_test_delayed_fill.argtypes = [C.c_void_p, C.c_void_p, C.c_double, C.c_int64,
                                               C.c_int]
    assert L.arpack_hip_test_delayed_fill(dst, src, value, count, DELAY_US) == 0


def _solve(pkg, A, v0=None):
    s = pkg.SymRci(N, NEV, NCV, "LA", 1e-10, mxiter=300, v0=v0, device=True)
    assert s.aupd_csr(A) == 99 and int(s.info[0]) == 0
    return s


@pytest.fixture(scope="module")
def op(pkg):
    return pkg.CSR.banded_sym(N, 77, 256, 12)


def test_aupd_waits_for_callers_resid(pkg, op):
    v0 = np.random.default_rng(3).standard_normal(N)
    ref = _solve(pkg, op, v0)
    src = pkg.DeviceBuffer.from_numpy(v0)
    s = pkg.SymRci(N, NEV, NCV, "LA", 1e-10, mxiter=300, device=True)
    s.info[0] = 1                      # the caller supplies resid ...
    _fill(pkg, s.resid.ptr, src.ptr, 0.0, N)   # ... with GPU work still in flight
    # witness: a null-stream read does not order behind it, so the race is real
    assert not np.any(s.resid.numpy(0, 1024))
    assert s.aupd_csr(op) == 99 and int(s.info[0]) == 0
    np.testing.assert_array_equal(s.iparam, ref.iparam)
    np.testing.assert_array_equal(s.ritz, ref.ritz)


def test_eupd_waits_for_callers_z(pkg, op):
    v0 = np.random.default_rng(4).standard_normal(N)
    a, b = _solve(pkg, op, v0), _solve(pkg, op, v0)
    d1, z1, nconv = a.eupd()
    zb = pkg.DeviceBuffer(NEV * N)
    _fill(pkg, zb.ptr, None, 1.0e300, NEV * N)  # the caller's late overwrite of Z
    d2, z2, nconv2 = b.eupd(z=zb)
    assert nconv2 == nconv == NEV
    np.testing.assert_array_equal(d2, d1)
    np.testing.assert_array_equal(zb.numpy(), z1.numpy())


def test_eupd_z_aliasing_v_waits(pkg, op):
    """Z = V (the reference's drivers pass v for z) while the caller's own GPU
    work still rewrites V's leading columns with the values they hold (a late
    identity write): eupd must run after it, so the Ritz vectors it leaves in
    V(:, 1:nconv) are the synchronous run's, not the old basis columns."""
    v0 = np.random.default_rng(5).standard_normal(N)
    a, b = _solve(pkg, op, v0), _solve(pkg, op, v0)
    _, za, nconv = a.eupd(z=a.v)
    lead = pkg.DeviceBuffer.from_numpy(b.v.numpy(0, NEV * b.ldv))
    _fill(pkg, b.v.ptr, lead.ptr, 0.0, NEV * b.ldv)
    _, zb, _ = b.eupd(z=b.v)
    ra = za.numpy().reshape(NCV, a.ldv)[:nconv, :N]
    rb = zb.numpy().reshape(NCV, b.ldv)[:nconv, :N]
    np.testing.assert_array_equal(rb, ra)


def test_csr_spmv_waits_for_callers_x(pkg, op):
    x = np.random.default_rng(6).standard_normal(N)
    xs = pkg.DeviceBuffer.from_numpy(x)
    ys = pkg.DeviceBuffer(N)
    op.matvec_device(xs, ys)
    src = pkg.DeviceBuffer.from_numpy(x)
    xa = pkg.DeviceBuffer(N)
    ya = pkg.DeviceBuffer(N)
    _fill(pkg, xa.ptr, src.ptr, 0.0, N)
    assert not np.any(xa.numpy(0, 1024))  # witness: still being written
    op.matvec_device(xa, ya)
    np.testing.assert_array_equal(ya.numpy(), ys.numpy())
