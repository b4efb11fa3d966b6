"""arpack-ng_amd — MI355X-native implicitly restarted Lanczos/Arnoldi behind
arpack-ng's reverse-communication interface.

The product is the C-ABI library ``libarpack_hip.so`` (declared in
``include/arpack_hip.h``).  This module is the Python host-side mirror of the
reference's interface for the path: thin ctypes bindings with the reference's
names and argument meaning (``dsaupd``/``dseupd`` behave like the Fortran
routines of SRC/dsaupd.f / SRC/dseupd.f, driven exactly like
TESTS/icb_arpack_c.c does), plus the native extension (device CSR operators and
the on-GPU driver).

There is no CPU fallback: if the HIP library is missing, every entry point
raises.  Device-pointer mode uses buffers allocated through the engine's own
HIP runtime (DeviceBuffer); PyTorch is only used for torch.distributed (gloo)
control traffic in the multi-process launcher.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from functools import partial

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ARPACK_HIP_LIB: load another build of the library (same-box A/B of build variants)
LIB_PATH = os.environ.get("ARPACK_HIP_LIB") or os.path.join(HERE, "libarpack_hip.so")

_lib = None


class ArpackError(RuntimeError):
    """Raised for negative `info` codes (SRC/dsaupd.f:243-276)."""

    def __init__(self, routine, info, extra=None):
        super().__init__(f"{routine} returned info={info}")
        self.routine = routine
        self.info = info
        self.extra = extra or {}


def build(jobs: int = 8) -> str:
    """Compile libarpack_hip.so for gfx950 in-tree (hipcc, no GPU needed)."""
    subprocess.run(["make", "-C", HERE, f"-j{jobs}"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} not built: the HIP engine is required (no CPU fallback); "
                "run arpack_ng_amd.build() / `make -C arpack-ng_amd`")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


_I = C.c_int
_PI = C.POINTER(C.c_int)
_PD = C.c_void_p  # double* (host or device)


def _declare(L):
    L.arpack_hip_version.restype = C.c_char_p
    L.arpack_hip_device_count.restype = C.c_int
    L.dsaupd_c.argtypes = [_PI, C.c_char_p, _I, C.c_char_p, _I, C.c_double, _PD, _I, _PD, _I,
                           _PI, _PI, _PD, _PD, _I, _PI]
    L.dseupd_c.argtypes = [_I, C.c_char_p, _PI, _PD, _PD, _I, C.c_double, C.c_char_p, _I,
                           C.c_char_p, _I, C.c_double, _PD, _I, _PD, _I, _PI, _PI, _PD, _PD, _I,
                           _PI]
    L.arpack_hip_dsaupd_csr.argtypes = [C.c_void_p] + L.dsaupd_c.argtypes
    L.arpack_hip_csr_create.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int64, C.c_void_p,
                                        C.c_void_p, C.c_void_p]
    L.arpack_hip_csr_destroy.argtypes = [C.c_void_p]
    L.arpack_hip_csr_spmv.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.arpack_hip_csr_set_kernel.argtypes = [C.c_void_p, C.c_int, C.c_int]
    L.arpack_hip_csr_set_symmetric.argtypes = [C.c_void_p, C.c_int]
    L.arpack_hip_csr_time.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    L.arpack_hip_csr_time.restype = C.c_double
    L.arpack_hip_csr_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.arpack_hip_csr_download.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.arpack_hip_gen_laplace2d.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_double]
    L.arpack_hip_gen_laplace3d.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_double]
    L.arpack_hip_gen_laplace3d_rows.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int64,
                                                C.c_int64, C.c_double]
    L.arpack_hip_gen_anderson.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int, C.c_double,
                                          C.c_uint32]
    L.arpack_hip_gen_banded_sym.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int64,
                                            C.c_int64, C.c_uint32, C.c_int, C.c_int]
    L.arpack_hip_set_stream.argtypes = [C.c_void_p]
    L.arpack_hip_fault_inject.argtypes = [C.c_long]
    L.arpack_hip_set_deterministic.argtypes = [C.c_int]
    L.arpack_hip_deterministic.restype = C.c_int
    L.arpack_hip_malloc.argtypes = [C.c_size_t]
    L.arpack_hip_malloc.restype = C.c_void_p
    L.arpack_hip_free.argtypes = [C.c_void_p]
    L.arpack_hip_memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.arpack_hip_memset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
    L.dsaupd_.argtypes = [_PI, C.c_char_p, _PI, C.c_char_p, _PI, C.POINTER(C.c_double), _PD, _PI,
                          _PD, _PI, _PI, _PI, _PD, _PD, _PI, _PI, C.c_size_t, C.c_size_t]
    L.stat_c.argtypes = [_PI] * 5 + [C.POINTER(C.c_float)] * 26
    L.arpack_hip_dsaupd_csr_cycles.argtypes = [C.c_void_p, _I, _PI, C.c_char_p, _I, C.c_char_p, _I,
                                               C.POINTER(C.c_double), _PD, _I, _PD, _I, _PI, _PI,
                                               _PD, _PD, _I, _PI]
    L.dnaupd_c.argtypes = L.dsaupd_c.argtypes
    L.dneupd_c.argtypes = [_I, C.c_char_p, _PI, _PD, _PD, _PD, _I, C.c_double, C.c_double, _PD,
                           C.c_char_p, _I, C.c_char_p, _I, C.c_double, _PD, _I, _PD, _I, _PI, _PI,
                           _PD, _PD, _I, _PI]
    L.dnaupd_.argtypes = L.dsaupd_.argtypes
    L.arpack_hip_dnaupd_csr_cycles.argtypes = L.arpack_hip_dsaupd_csr_cycles.argtypes
    L.arpack_hip_dsaupd_shift.argtypes = [C.c_void_p, _PI, C.c_char_p, _I, C.c_char_p, _I,
                                          C.POINTER(C.c_double), _PD, _I, _PD, _I, _PI, _PI,
                                          _PD, _PD, _I, _PI]
    L.arpack_hip_dnaupd_shift.argtypes = L.arpack_hip_dsaupd_shift.argtypes
    L.arpack_hip_gen_convdiff2d.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_double]
    L.znaupd_c.argtypes = [_PI, C.c_char_p, _I, C.c_char_p, _I, C.c_double, _PD, _I, _PD, _I,
                           _PI, _PI, _PD, _PD, _I, _PD, _PI]
    L.arpack_hip_znaupd_zcsr.argtypes = [C.c_void_p, _PI, C.c_char_p, _I, C.c_char_p, _I,
                                         C.POINTER(C.c_double), _PD, _I, _PD, _I, _PI, _PI, _PD,
                                         _PD, _I, _PD, _PI]
    L.arpack_hip_zcsr_create.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int64, C.c_void_p,
                                         C.c_void_p, C.c_void_p]
    L.arpack_hip_gen_zrandom.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int, C.c_uint32,
                                         C.c_double]
    L.arpack_hip_zcsr_destroy.argtypes = [C.c_void_p]
    L.arpack_hip_zcsr_info.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.arpack_hip_zcsr_download.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.arpack_hip_zcsr_spmv.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.arpack_hip_zshift_create.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_double,
                                           C.c_double, C.c_double, _I]
    L.arpack_hip_zshift_destroy.argtypes = [C.c_void_p]
    L.arpack_hip_zshift_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, _PD]
    L.arpack_hip_zshift_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_longlong)] * 3 + [_PD] * 3
    L.arpack_hip_znaupd_zshift.argtypes = L.arpack_hip_znaupd_zcsr.argtypes
    L.arpack_hip_dshift_create.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_double,
                                           C.c_double, _I]
    L.arpack_hip_dshift_destroy.argtypes = [C.c_void_p]
    L.arpack_hip_dshift_set_method.argtypes = [C.c_void_p, _I]
    L.arpack_hip_dshift_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, _PD]
    L.arpack_hip_dshift_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_longlong)] * 3 + [_PD] * 3
    L.arpack_hip_profile.argtypes = [_I]
    L.arpack_hip_profile_read.argtypes = [_PD, _PD, _PD, _I]
    L.arpack_hip_synchronize.restype = C.c_int
    L.arpack_hip_kit_dstqrb.argtypes = [_I, _PD, _PD, _PD, _PD]
    L.arpack_hip_kit_dsteqr.argtypes = [_I, _PD, _PD, _PD, _I, _PD]
    L.arpack_hip_kit_dlartg.argtypes = [C.c_double, C.c_double] + [C.POINTER(C.c_double)] * 3
    L.arpack_hip_kit_dsortr.argtypes = [C.c_char_p, _I, _I, _PD, _PD]
    L.arpack_hip_kit_dsapps_host.argtypes = [_I, _I, _PD, _PD, _I, _PD, _I]
    L.arpack_hip_kit_dlarnv.argtypes = [_PI, _I, _PD]
    L.arpack_hip_kit_slarnv.argtypes = [_PI, _I, _PD]
    # single-precision family: the d* signatures with float tol / sigma
    def _f32(args, idx):
        a = list(args)
        for i in idx:
            a[i] = C.c_float if a[i] is C.c_double else C.POINTER(C.c_float)
        return a
    L.ssaupd_c.argtypes = _f32(L.dsaupd_c.argtypes, [5])
    L.snaupd_c.argtypes = _f32(L.dnaupd_c.argtypes, [5])
    L.ssaupd_.argtypes = _f32(L.dsaupd_.argtypes, [5])
    L.snaupd_.argtypes = _f32(L.dnaupd_.argtypes, [5])
    L.sseupd_c.argtypes = _f32(L.dseupd_c.argtypes, [6, 11])
    L.sneupd_c.argtypes = _f32(L.dneupd_c.argtypes, [7, 8, 14])


def version() -> str:
    return lib().arpack_hip_version().decode()


def device_count() -> int:
    return lib().arpack_hip_device_count()


def pci_bus_id(device: int = 0) -> str:
    """PCI bus id of a device (arpack_hip_device_pci_bus_id); "" if unknown."""
    buf = C.create_string_buffer(64)
    L = lib()
    L.arpack_hip_device_pci_bus_id.argtypes = [C.c_int, C.c_char_p, C.c_int]
    if L.arpack_hip_device_pci_bus_id(int(device), buf, 64) != 0:
        return ""
    return buf.value.decode()


# ----------------------------------------------------------------------------- arrays
class DeviceBuffer:
    """A float64 buffer in HBM, allocated through the engine's own HIP runtime
    (arpack_hip_malloc), so no second GPU runtime is needed in the process."""

    def __init__(self, n, dtype=np.float64):
        self.dtype = np.dtype(dtype)
        self.n = int(n)
        self.nbytes = self.n * self.dtype.itemsize
        self.ptr = lib().arpack_hip_malloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"arpack_hip_malloc({self.nbytes}) failed")
        lib().arpack_hip_memset(self.ptr, 0, self.nbytes)

    @classmethod
    def from_numpy(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.size, a.dtype)
        lib().arpack_hip_memcpy(b.ptr, a.ctypes.data, b.nbytes)
        return b

    def numpy(self, offset=0, count=None):
        count = self.n - offset if count is None else count
        out = np.empty(count, self.dtype)
        lib().arpack_hip_memcpy(out.ctypes.data, self.ptr + offset * self.dtype.itemsize,
                                count * self.dtype.itemsize)
        return out

    def write(self, a, offset=0):
        a = np.ascontiguousarray(a, self.dtype)
        lib().arpack_hip_memcpy(self.ptr + offset * self.dtype.itemsize, a.ctypes.data, a.nbytes)

    def at(self, offset):
        """Device address of element `offset`."""
        return self.ptr + offset * self.dtype.itemsize

    def __len__(self):
        return self.n

    def __del__(self):
        try:
            if self.ptr and _lib is not None:
                _lib.arpack_hip_free(self.ptr)
                self.ptr = None
        except Exception:
            pass


def _ptr(a):
    """Raw address of a numpy array (host) or a DeviceBuffer / torch tensor (device)."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if isinstance(a, DeviceBuffer):
        return a.ptr
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    raise TypeError(type(a))


def _ip(a):
    return a.ctypes.data_as(_PI)


PROF_CLASSES = ["spmv", "cgs_dots", "update", "vq", "place", "finalize", "other", "allreduce",
                "halo"]


def profile(enable: bool = True):
    """Turn the engine's per-kernel hipEvent timing on/off."""
    lib().arpack_hip_profile(1 if enable else 0)


def profile_read():
    """{class: (total_ms, algorithmic_bytes, launches)} since the last read."""
    k = len(PROF_CLASSES)
    ms = np.zeros(k)
    by = np.zeros(k)
    cnt = np.zeros(k, np.int64)
    lib().arpack_hip_profile_read(ms.ctypes.data, by.ctypes.data, cnt.ctypes.data, k)
    return {c: (float(ms[i]), float(by[i]), int(cnt[i])) for i, c in enumerate(PROF_CLASSES)}


def set_deterministic(on: bool = True):
    """Deterministic mode (arpack_hip_set_deterministic): only fixed-order SpMV
    forms, so solves are bitwise reproducible run to run.  Set it before
    CSR.set_symmetric (which then keeps full storage)."""
    lib().arpack_hip_set_deterministic(1 if on else 0)


def deterministic() -> bool:
    return bool(lib().arpack_hip_deterministic())


def fault_inject(k: int):
    """Test hook: the k-th checked HIP call of the engine from now on reports
    hipErrorInvalidValue (arpack_hip_fault_inject); 0 disarms."""
    lib().arpack_hip_fault_inject(int(k))


def synchronize():
    if lib().arpack_hip_synchronize() != 0:
        raise RuntimeError("hipDeviceSynchronize failed")


def stats():
    """stat_c(): /timing/ counters of the last solve (stat.h:8-21)."""
    L = lib()
    ints = [C.c_int() for _ in range(5)]
    fl = [C.c_float() for _ in range(26)]
    L.stat_c(*[C.byref(i) for i in ints], *[C.byref(f) for f in fl])
    return dict(zip(["nopx", "nbx", "nrorth", "nitref", "nrstrt"], [i.value for i in ints]))


# ------------------------------------------------------------------- CSR operator
class CSR:
    """A CSR matrix resident in HBM (the `ido=+-1` OP served on the GPU)."""

    def __init__(self, handle, owner=True):
        self.h = C.c_void_p(handle)
        n = C.c_int64()
        nnz = C.c_int64()
        lib().arpack_hip_csr_info(self.h, C.byref(n), C.byref(nnz))
        self.n, self.nnz = n.value, nnz.value
        self._owner = owner

    def __del__(self):
        try:
            if self._owner and self.h and _lib is not None:
                _lib.arpack_hip_csr_destroy(self.h)
                self.h = C.c_void_p(0)
        except Exception:
            pass

    @classmethod
    def from_arrays(cls, rowptr, col, val):
        rowptr = np.ascontiguousarray(rowptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        val = np.ascontiguousarray(val, np.float64)
        h = C.c_void_p()
        rc = lib().arpack_hip_csr_create(C.byref(h), len(rowptr) - 1, len(col), rowptr.ctypes.data,
                                         col.ctypes.data, val.ctypes.data)
        if rc != 0:
            raise RuntimeError("arpack_hip_csr_create failed")
        return cls(h.value)

    @classmethod
    def laplace2d(cls, m, scale=1.0):
        h = C.c_void_p()
        if lib().arpack_hip_gen_laplace2d(C.byref(h), m, scale) != 0:
            raise RuntimeError("laplace2d generation failed")
        return cls(h.value)

    @classmethod
    def convdiff2d(cls, m, rho):
        """-Lap u + rho du/dx (EXAMPLES/NONSYM/dndrv1.f:397-475), m x m grid."""
        h = C.c_void_p()
        if lib().arpack_hip_gen_convdiff2d(C.byref(h), m, rho) != 0:
            raise RuntimeError("convdiff2d generation failed")
        return cls(h.value)

    @classmethod
    def laplace3d(cls, m, scale=1.0, r0=0, r1=None):
        """The m^3 7-pt Laplacian (BASELINE config 4); with r0/r1, only rows
        [r0, r1) with global columns -- one rank's z-slab block for DistOp
        (arpack_hip_gen_laplace3d_rows)."""
        h = C.c_void_p()
        if r0 == 0 and r1 is None:
            rc = lib().arpack_hip_gen_laplace3d(C.byref(h), m, scale)
        else:
            rc = lib().arpack_hip_gen_laplace3d_rows(C.byref(h), m, r0, m ** 3 if r1 is None else r1,
                                                     scale)
        if rc != 0:
            raise RuntimeError("laplace3d generation failed (rc=%d)" % rc)
        return cls(h.value)

    @classmethod
    def anderson(cls, m, dim=3, disorder=16.0, seed=1234):
        h = C.c_void_p()
        if lib().arpack_hip_gen_anderson(C.byref(h), m, dim, disorder, seed) != 0:
            raise RuntimeError("anderson generation failed")
        return cls(h.value)

    @classmethod
    def banded_sym(cls, n, seed=1234, bandwidth=4096, per_row=25, r0=0, r1=None):
        h = C.c_void_p()
        r1 = n if r1 is None else r1
        if lib().arpack_hip_gen_banded_sym(C.byref(h), n, r0, r1, seed, bandwidth, per_row) != 0:
            raise RuntimeError("banded_sym generation failed")
        return cls(h.value)

    def download(self):
        rowptr = np.empty(self.n + 1, np.int64)
        col = np.empty(self.nnz, np.int32)
        val = np.empty(self.nnz, np.float64)
        lib().arpack_hip_csr_download(self.h, rowptr.ctypes.data, col.ctypes.data, val.ctypes.data)
        return rowptr, col, val

    def set_kernel(self, kernel: int, tile: int = 4096):
        """0 vector, 1 CSR-stream, 2 CSR-stream non-temporal."""
        if lib().arpack_hip_csr_set_kernel(self.h, kernel, tile) != 0:
            raise RuntimeError("kernel not applicable to this matrix")

    def set_symmetric(self, on: bool = True):
        """Declare the matrix symmetric: the SpMV streams only the upper
        triangle (arpack_hip_csr_set_symmetric; entries below the diagonal are
        ignored).  Raises if the band structure does not fit the LDS windows.
        On one rank's block of a DistOp the call is collective: every rank
        must make it, and all raise (full storage kept) if any rank's plan
        fails -- rc = -2 on the ranks whose own plan succeeded."""
        rc = lib().arpack_hip_csr_set_symmetric(self.h, 1 if on else 0)
        self.last_rc = rc
        if rc == 1:  # deterministic mode: the full-storage (fixed-order) SpMV stays
            self.symmetric = False
            return
        if rc != 0:
            raise RuntimeError("symmetric storage not applicable to this matrix (rc=%d)" % rc)
        self.symmetric = bool(on)

    def set_sym_accumulator(self, acc: str = "fixed"):
        """The symmetric kernel's transposed-term accumulator: "fixed" (the
        fixed-point form, bitwise reproducible; default) or "fp64" (LDS fp64
        atomics in schedule order) -- arpack_hip_csr_set_sym_accumulator."""
        lib().arpack_hip_csr_set_sym_accumulator.argtypes = [C.c_void_p, C.c_int]
        if lib().arpack_hip_csr_set_sym_accumulator(self.h, {"fixed": 0, "fp64": 1}[acc]) != 0:
            raise RuntimeError("set_sym_accumulator failed")

    @property
    def sym_form(self):
        """"full", "sym_fp64" or "sym_fixed": the SpMV form the operator runs
        now (arpack_hip_csr_sym_form)."""
        lib().arpack_hip_csr_sym_form.argtypes = [C.c_void_p]
        return ("full", "sym_fp64", "sym_fixed")[lib().arpack_hip_csr_sym_form(self.h)]

    def time_spmv(self, reps=20):
        x = DeviceBuffer(self.n)
        x.write(np.linspace(-1, 1, self.n))
        y = DeviceBuffer(self.n)
        return lib().arpack_hip_csr_time(self.h, x.ptr, y.ptr, reps)

    def matvec_device(self, x, y):
        """y = A x for device addresses (ints) or DeviceBuffers."""
        xp = x if isinstance(x, int) else _ptr(x)
        yp = y if isinstance(y, int) else _ptr(y)
        if lib().arpack_hip_csr_spmv(self.h, xp, yp) != 0:
            raise RuntimeError("spmv failed")


# ------------------------------------------------------------- RCI (reference API)
class SymRci:
    """State of one dsaupd/dseupd solve, mirroring the reference's argument list
    (SRC/dsaupd.f:182-186).  `device=True` allocates resid/V/workd in HBM
    (torch tensors) so the caller's OP works on device pointers; otherwise
    numpy host arrays (the engine mirrors them in HBM)."""

    _fam = "s"  # dsaupd / ssaupd

    def __init__(self, n, nev, ncv, which="LM", tol=0.0, bmat="I", mode=1, mxiter=300,
                 ishift=1, v0=None, device=False, icb=False, prec="d"):
        """prec="s": the single-precision family (ssaupd / snaupd): float32 arrays."""
        self.n, self.nev, self.ncv = n, nev, ncv
        self.icb = icb
        self.prec = prec
        self.dt = np.float32 if prec == "s" else np.float64
        self.which, self.bmat, self.tol = which, bmat, float(tol)
        self.device = device
        self.ido = np.zeros(1, np.int32)
        self.info = np.zeros(1, np.int32)
        self.iparam = np.zeros(11, np.int32)
        self.ipntr = np.zeros(11, np.int32)
        self.iparam[0] = ishift
        self.iparam[2] = mxiter
        self.iparam[6] = mode
        self.lworkl = ncv * ncv + 8 * ncv
        self.workl = np.zeros(self.lworkl, self.dt)
        # device V: columns padded to 128-B lines (ldv >= n, as ARPACK allows);
        # a column start off a line costs the Gram-Schmidt and V*Q passes 8-12%
        # (profiles/r03am_summary.txt: n = 10^7 - 1 against 10^7)
        # (ARPACK_HIP_LDV_PAD=0: ldv = n, for a same-box A/B)
        al = 128 // np.dtype(self.dt).itemsize
        pad = device and os.environ.get("ARPACK_HIP_LDV_PAD", "1") != "0"
        self.ldv = -(-n // al) * al if pad else n
        if device:
            self.resid = DeviceBuffer(n, self.dt)
            self.v = DeviceBuffer(ncv * self.ldv, self.dt)
            self.workd = DeviceBuffer(3 * n, self.dt)
            if v0 is not None:
                self.resid.write(np.asarray(v0, self.dt))
        else:
            self.resid = np.zeros(n, self.dt) if v0 is None else np.array(v0, self.dt, copy=True)
            self.v = np.zeros(ncv * n, self.dt)
            self.workd = np.zeros(3 * n, self.dt)
        self.info[0] = 0 if v0 is None else 1

    def aupd(self):
        """One dsaupd call (dnaupd for NsRci, s* for prec="s"); returns ido.  Uses
        the Fortran entry dsaupd_ (tol by reference, so tol <= 0 becomes eps for
        the rest of the solve exactly as in SRC/dsaupd.f:550) unless icb=True
        selects dsaupd_c (tol by value on every call, SRC/icbads.F90:14)."""
        name = self.prec + self._fam + "aupd_"
        if self.icb:
            getattr(lib(), name + "c")(
                _ip(self.ido), self.bmat.encode(), self.n, self.which.encode(), self.nev, self.tol,
                _ptr(self.resid), self.ncv, _ptr(self.v), self.ldv, _ip(self.iparam),
                _ip(self.ipntr), _ptr(self.workd), self.workl.ctypes.data, self.lworkl,
                _ip(self.info))
        else:
            tol = (C.c_float if self.prec == "s" else C.c_double)(self.tol)
            getattr(lib(), name)(
                _ip(self.ido), self.bmat.encode(), C.byref(C.c_int(self.n)), self.which.encode(),
                C.byref(C.c_int(self.nev)), C.byref(tol), _ptr(self.resid),
                C.byref(C.c_int(self.ncv)), _ptr(self.v), C.byref(C.c_int(self.ldv)),
                _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd), self.workl.ctypes.data,
                C.byref(C.c_int(self.lworkl)), _ip(self.info), 1, 2)
            self.tol = tol.value
        return int(self.ido[0])

    def aupd_csr(self, A: CSR):
        """Run to completion with OP = A on the GPU (arpack_hip_dsaupd_csr)."""
        lib().arpack_hip_dsaupd_csr(A.h, _ip(self.ido), self.bmat.encode(), self.n,
                                    self.which.encode(), self.nev, self.tol, _ptr(self.resid),
                                    self.ncv, _ptr(self.v), self.ldv, _ip(self.iparam),
                                    _ip(self.ipntr), _ptr(self.workd), self.workl.ctypes.data,
                                    self.lworkl, _ip(self.info))
        if self.tol <= 0.0:  # the solve used eps (SRC/dsaupd.f:550); keep it for dseupd
            self.tol = float(np.finfo(np.float64).eps / 2)
        return int(self.ido[0])

    def aupd_cycles(self, A: CSR, max_cycles: int):
        """Free-running solve that parks (ido=98) after `max_cycles` more restart
        cycles (arpack_hip_dsaupd_csr_cycles); returns ido (98 parked, 99 done)."""
        tol = C.c_double(self.tol)
        lib().arpack_hip_dsaupd_csr_cycles(A.h, int(max_cycles), _ip(self.ido), self.bmat.encode(),
                                           self.n, self.which.encode(), self.nev, C.byref(tol),
                                           _ptr(self.resid), self.ncv, _ptr(self.v), self.ldv,
                                           _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd),
                                           self.workl.ctypes.data, self.lworkl, _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def aupd_shift(self, S: "DShift"):
        """Whole loop on the GPU in mode 3 (construct with mode=3): OP =
        (A - sigma I)^{-1} by the device CG S (arpack_hip_dsaupd_shift)."""
        tol = C.c_double(self.tol)
        lib().arpack_hip_dsaupd_shift(S.h, _ip(self.ido), self.bmat.encode(), self.n,
                                      self.which.encode(), self.nev, C.byref(tol),
                                      _ptr(self.resid), self.ncv, _ptr(self.v), self.ldv,
                                      _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd),
                                      self.workl.ctypes.data, self.lworkl, _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def aupd_gen(self, G: "DGen"):
        """Whole loop on the GPU in a generalized mode (construct with bmat="G",
        mode=G.mode): OP*x and B*x by the device operator pair G
        (arpack_hip_dsaupd_gen)."""
        tol = C.c_double(self.tol)
        L = lib()
        L.arpack_hip_dsaupd_gen.argtypes = L.arpack_hip_dsaupd_shift.argtypes
        L.arpack_hip_dsaupd_gen(G.h, _ip(self.ido), self.bmat.encode(), self.n,
                                self.which.encode(), self.nev, C.byref(tol),
                                _ptr(self.resid), self.ncv, _ptr(self.v), self.ldv,
                                _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd),
                                self.workl.ctypes.data, self.lworkl, _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def slice(self, k):
        """workd slice ipntr[k] (1-based offset) of length n: a numpy view in
        host mode, the device address (int) in device mode."""
        o = int(self.ipntr[k]) - 1
        if isinstance(self.workd, DeviceBuffer):
            return self.workd.at(o)
        return self.workd[o:o + self.n]

    def eupd(self, rvec=True, howmny="A", sigma=0.0, z=None, dist=None):
        """dseupd_c, or arpack_hip_pdseupd_c on this rank's rows when `dist`
        (a DistRows / DistOp) is given."""
        nconv = int(self.iparam[4])
        d = np.zeros(self.nev, self.dt)
        if z is None:
            m = self.nev * self.n
            z = DeviceBuffer(m, self.dt) if self.device else np.zeros(m, self.dt)
        select = np.zeros(self.ncv, np.int32)
        info = np.zeros(1, np.int32)
        f = (getattr(lib(), self.prec + "seupd_c") if dist is None
             else partial(lib().arpack_hip_pdseupd_c, dist.h))
        ldz = self.ldv if z is self.v else self.n  # Z = V (the reference's drivers)
        f(1 if rvec else 0, howmny.encode(), _ip(select), d.ctypes.data, _ptr(z), ldz, sigma,
          self.bmat.encode(), self.n, self.which.encode(), self.nev, self.tol, _ptr(self.resid),
          self.ncv, _ptr(self.v), self.ldv, _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd),
          self.workl.ctypes.data, self.lworkl, _ip(info))
        if info[0] < 0:
            raise ArpackError("dseupd", int(info[0]))
        return d[:nconv], z, nconv

    @property
    def ritz(self):
        o = int(self.ipntr[5]) - 1
        return self.workl[o:o + self.ncv].copy()


class NsRci(SymRci):
    """dnaupd state (SRC/dnaupd.f:400-693): like SymRci, with ipntr(14) and
    lworkl = 3*ncv^2 + 6*ncv; Ritz values are complex (ritzr/ritzi)."""

    _fam = "n"  # dnaupd / snaupd

    def __init__(self, n, nev, ncv, which="LM", tol=0.0, bmat="I", mode=1, mxiter=300,
                 ishift=1, v0=None, device=False, icb=False, prec="d"):
        super().__init__(n, nev, ncv, which, tol, bmat, mode, mxiter, ishift, v0, device, icb,
                         prec)
        self.ipntr = np.zeros(14, np.int32)
        self.lworkl = 3 * ncv * ncv + 6 * ncv
        self.workl = np.zeros(self.lworkl, self.dt)

    def aupd_cycles(self, A: CSR, max_cycles: int):
        tol = C.c_double(self.tol)
        lib().arpack_hip_dnaupd_csr_cycles(A.h, int(max_cycles), _ip(self.ido), self.bmat.encode(),
                                           self.n, self.which.encode(), self.nev, C.byref(tol),
                                           _ptr(self.resid), self.ncv, _ptr(self.v), self.ldv,
                                           _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd),
                                           self.workl.ctypes.data, self.lworkl, _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def aupd_gen(self, G: "DGen"):
        """Whole loop on the GPU in dnaupd's generalized modes (bmat="G", mode
        2, or 3 with G's real sigma): OP*x and B*x by the device operator pair
        G (arpack_hip_dnaupd_gen)."""
        tol = C.c_double(self.tol)
        L = lib()
        L.arpack_hip_dnaupd_gen.argtypes = L.arpack_hip_dsaupd_shift.argtypes
        L.arpack_hip_dnaupd_gen(G.h, _ip(self.ido), self.bmat.encode(), self.n,
                                self.which.encode(), self.nev, C.byref(tol),
                                _ptr(self.resid), self.ncv, _ptr(self.v), self.ldv,
                                _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd),
                                self.workl.ctypes.data, self.lworkl, _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def aupd_shift(self, S: "DShift"):
        """dnaupd in mode 3 (real shift) with OP = (A - sigma I)^{-1} by the
        device BiCGStab S (arpack_hip_dnaupd_shift)."""
        tol = C.c_double(self.tol)
        lib().arpack_hip_dnaupd_shift(S.h, _ip(self.ido), self.bmat.encode(), self.n,
                                      self.which.encode(), self.nev, C.byref(tol),
                                      _ptr(self.resid), self.ncv, _ptr(self.v), self.ldv,
                                      _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd),
                                      self.workl.ctypes.data, self.lworkl, _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def aupd_csr(self, A: CSR):
        r = self.aupd_cycles(A, -1)
        if self.tol <= 0.0:
            self.tol = float(np.finfo(np.float64).eps / 2)
        return r

    def eupd(self, rvec=True, howmny="A", sigmar=0.0, sigmai=0.0, z=None, dist=None):
        """dneupd_c: returns (dr, di, Z, nconv); Z has nev+1 columns (SRC/dneupd.f)."""
        nconv = int(self.iparam[4])
        dr, di = np.zeros(self.nev + 1, self.dt), np.zeros(self.nev + 1, self.dt)
        if z is None:
            m = (self.nev + 1) * self.n
            z = DeviceBuffer(m, self.dt) if self.device else np.zeros(m, self.dt)
        select = np.zeros(self.ncv, np.int32)
        workev = np.zeros(3 * self.ncv, self.dt)
        info = np.zeros(1, np.int32)
        f = (getattr(lib(), self.prec + "neupd_c") if dist is None
             else partial(lib().arpack_hip_pdneupd_c, dist.h))
        ldz = self.ldv if z is self.v else self.n  # Z = V (the reference's drivers)
        f(1 if rvec else 0, howmny.encode(), _ip(select), dr.ctypes.data, di.ctypes.data, _ptr(z),
          ldz, sigmar, sigmai, workev.ctypes.data, self.bmat.encode(), self.n,
          self.which.encode(), self.nev, self.tol, _ptr(self.resid), self.ncv, _ptr(self.v),
          self.ldv, _ip(self.iparam), _ip(self.ipntr), _ptr(self.workd), self.workl.ctypes.data,
          self.lworkl, _ip(info))
        if info[0] < 0:
            raise ArpackError("dneupd", int(info[0]))
        self.eupd_info = int(info[0])
        return dr[:nconv], di[:nconv], z, nconv

    @property
    def ritz(self):
        o, oi = int(self.ipntr[5]) - 1, int(self.ipntr[6]) - 1
        return self.workl[o:o + self.ncv] + 1j * self.workl[oi:oi + self.ncv]


class ZCSR:
    """Complex CSR operator in HBM (arpack_hip_zcsr)."""

    def __init__(self, handle):
        self.h = handle
        n, nnz = C.c_int64(), C.c_int64()
        lib().arpack_hip_zcsr_info(self.h, C.byref(n), C.byref(nnz))
        self.n, self.nnz = n.value, nnz.value

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.arpack_hip_zcsr_destroy(self.h)
        except Exception:
            pass

    @classmethod
    def from_arrays(cls, rowptr, col, val):
        rp = np.ascontiguousarray(rowptr, np.int64)
        cc = np.ascontiguousarray(col, np.int32)
        vv = np.ascontiguousarray(val, np.complex128)
        h = C.c_void_p()
        if lib().arpack_hip_zcsr_create(C.byref(h), len(rp) - 1, len(cc), rp.ctypes.data,
                                        cc.ctypes.data, vv.ctypes.data) != 0:
            raise RuntimeError("zcsr_create failed")
        return cls(h.value)

    def tile_info(self):
        """(form, stored): the product's layout (arpack_hip_zcsr_tile_info: 0
        CSR, 1 slice CSRs, 2 sorted tiles, 3 packed tiles) and entries streamed."""
        L = lib()
        L.arpack_hip_zcsr_tile_info.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int64)]
        f, st = C.c_int(), C.c_int64()
        L.arpack_hip_zcsr_tile_info(self.h, C.byref(f), C.byref(st))
        return f.value, st.value

    @classmethod
    def random(cls, n, per_row=100, seed=5, dshift=100.0):
        """BASELINE config 5 operator generated in HBM (oracle twin: matrices.zrandom)."""
        h = C.c_void_p()
        if lib().arpack_hip_gen_zrandom(C.byref(h), n, per_row, seed, dshift) != 0:
            raise RuntimeError("gen_zrandom failed")
        return cls(h.value)

    def matvec(self, x):
        """y = A x for a host complex vector (through HBM; arpack_hip_zcsr_spmv --
        the XCD column-split kernel when the operator qualifies)."""
        xv = np.ascontiguousarray(x, np.complex128).view(np.float64)
        xb, yb = DeviceBuffer(2 * self.n), DeviceBuffer(2 * self.n)
        xb.write(xv)
        if lib().arpack_hip_zcsr_spmv(self.h, _ptr(xb), _ptr(yb)) != 0:
            raise RuntimeError("zcsr spmv failed")
        return yb.numpy().view(np.complex128).copy()

    def download(self):
        rp = np.zeros(self.n + 1, np.int64)
        col = np.zeros(self.nnz, np.int32)
        val = np.zeros(self.nnz, np.complex128)
        lib().arpack_hip_zcsr_download(self.h, rp.ctypes.data, col.ctypes.data, val.ctypes.data)
        return rp, col, val


class ZShift:
    """Shift-invert operator y = (A - sigma I)^{-1} x on the GPU (BiCGStab over the
    complex CSR operator; arpack_hip_zshift_*): znaupd's mode-3 OP (SRC/znaupd.f:27),
    the caller-side solve the reference's drivers do with zgttrf/zgttrs
    (EXAMPLES/COMPLEX/zndrv2.f:179,250)."""

    def __init__(self, A: "ZCSR", sigma=0j, rtol=1e-12, maxit=200, method="bicgstab"):
        """method: "bicgstab", or "tridiag" (a direct solve of a tridiagonal
        A - sigma I: zgttrf + device scans, as zndrv2.f's zgttrf / zgttrs)."""
        self.A = A  # keeps the operator alive
        self.sigma = complex(sigma)
        h = C.c_void_p()
        rc = lib().arpack_hip_zshift_create(C.byref(h), A.h, self.sigma.real, self.sigma.imag,
                                            float(rtol), int(maxit))
        if rc != 0:
            raise RuntimeError("arpack_hip_zshift_create failed (%d)" % rc)
        self.h = h.value
        self.n = A.n
        if method != "bicgstab":
            L = lib()
            L.arpack_hip_zshift_set_method.argtypes = [C.c_void_p, C.c_int]
            if L.arpack_hip_zshift_set_method(self.h, {"tridiag": 1}[method]) != 0:
                raise ValueError(method)

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.arpack_hip_zshift_destroy(self.h)
        except Exception:
            pass

    def solve(self, x):
        """y = (A - sigma I)^{-1} x for a host complex vector; returns (y, iters, relres)."""
        xv = np.ascontiguousarray(x, np.complex128).view(np.float64)
        xb, yb = DeviceBuffer(2 * self.n), DeviceBuffer(2 * self.n)
        xb.write(xv)
        rr = C.c_double()
        it = lib().arpack_hip_zshift_solve(self.h, _ptr(xb), _ptr(yb), C.byref(rr))
        if it == -2:
            raise RuntimeError("zshift solve: HIP error")
        return yb.numpy().view(np.complex128).copy(), it, rr.value

    def stats(self):
        a, b, c = C.c_longlong(), C.c_longlong(), C.c_longlong()
        d, e, f = C.c_double(), C.c_double(), C.c_double()
        lib().arpack_hip_zshift_stats(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d),
                                      C.byref(e), C.byref(f))
        return dict(solves=a.value, iters=b.value, failures=c.value, max_relres=d.value,
                    ms=e.value, bytes_per_iter=f.value)


class DShift:
    """Shift-invert operator y = (A - sigma I)^{-1} x on the GPU for a symmetric CSR
    operator (conjugate gradients or MINRES; arpack_hip_dshift_*): dsaupd's mode-3
    OP (SRC/dsaupd.f:30-48), the caller-side solve EXAMPLES/SYM/dsdrv2.f does with
    dgttrf/dgttrs."""

    def __init__(self, A: "CSR", sigma=0.0, rtol=1e-12, maxit=1000, method="cg"):
        """method: "cg" (A - sigma I positive definite), "minres" (any symmetric
        A - sigma I, e.g. sigma inside the spectrum), "bicgstab" (a nonsymmetric
        A: dnaupd's real shift-invert) or "tridiag" (a direct solve of a
        tridiagonal A - sigma I: dgttrf + device scans)."""
        self.A = A  # keeps the operator alive
        self.sigma = float(sigma)
        h = C.c_void_p()
        rc = lib().arpack_hip_dshift_create(C.byref(h), A.h, self.sigma, float(rtol), int(maxit))
        if rc != 0:
            raise RuntimeError("arpack_hip_dshift_create failed (%d)" % rc)
        self.h = h.value
        self.n = A.n
        if lib().arpack_hip_dshift_set_method(self.h, {"cg": 0, "minres": 1, "bicgstab": 2,
                                                       "tridiag": 3}[method]) != 0:
            raise ValueError(method)

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.arpack_hip_dshift_destroy(self.h)
        except Exception:
            pass

    def solve(self, x):
        """y = (A - sigma I)^{-1} x for a host vector; returns (y, iters, relres)."""
        xb, yb = DeviceBuffer(self.n), DeviceBuffer(self.n)
        xb.write(np.ascontiguousarray(x, np.float64))
        rr = C.c_double()
        it = lib().arpack_hip_dshift_solve(self.h, _ptr(xb), _ptr(yb), C.byref(rr))
        if it == -2:
            raise RuntimeError("dshift solve: HIP error")
        return yb.numpy().copy(), it, rr.value

    def stats(self):
        a, b, c = C.c_longlong(), C.c_longlong(), C.c_longlong()
        d, e, f = C.c_double(), C.c_double(), C.c_double()
        lib().arpack_hip_dshift_stats(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d),
                                      C.byref(e), C.byref(f))
        return dict(solves=a.value, iters=b.value, failures=c.value, max_relres=d.value,
                    ms=e.value, bytes_per_iter=f.value)



class DGen:
    """Device operator pair of dsaupd's generalized modes (bmat = 'G', modes
    2-5; arpack_hip_dgen_create): mode 2 OP = inv[M] A; 3 OP = inv[A - sigma M]
    M; 4 (buckling, A = K, B = KG) OP = inv[K - sigma KG] K; 5 (Cayley) OP =
    inv[A - sigma M](A + sigma M).  The inverse is a device CG (method 0),
    MINRES (1) or BiCGStab (2: a nonsymmetric C, dnaupd's modes 2-3 through
    NsRci.aupd_gen) to relative residual rtol on C = A - sigma B."""

    def __init__(self, A: CSR, B: CSR, mode: int, sigma=0.0, rtol: float = 1e-12,
                 maxit: int = 5000, method: int = 0):
        """A complex sigma (nonzero imaginary part): dnaupd's complex-shift
        modes 3 / 4 (OP = Re / Im of inv[A - sigma M] M; method 2 BiCGStab or 3
        the direct tridiagonal solve, on the complex C)."""
        L = lib()
        L.arpack_hip_dgen_create.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_int,
                                             C.c_double, C.c_double, C.c_int, C.c_int]
        L.arpack_hip_dgen_create_cshift.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p,
                                                    C.c_int, C.c_double, C.c_double, C.c_double,
                                                    C.c_int, C.c_int]
        L.arpack_hip_dgen_destroy.argtypes = [C.c_void_p]
        h = C.c_void_p()
        sigma = complex(sigma)
        if sigma.imag != 0.0:
            rc = L.arpack_hip_dgen_create_cshift(C.byref(h), A.h, B.h, int(mode), sigma.real,
                                                 sigma.imag, float(rtol), int(maxit),
                                                 {2: 0, 3: 1}[int(method)])
        else:
            rc = L.arpack_hip_dgen_create(C.byref(h), A.h, B.h, int(mode), sigma.real, float(rtol),
                                          int(maxit), int(method))
        if rc != 0:
            raise RuntimeError(f"arpack_hip_dgen_create failed ({rc})")
        self.h, self.A, self.B, self.mode = h, A, B, int(mode)

    def stats(self):
        L = lib()
        L.arpack_hip_dgen_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_longlong)] * 3 + [_PD]
        v = [C.c_longlong() for _ in range(3)]
        r = C.c_double()
        L.arpack_hip_dgen_stats(self.h, *[C.byref(x) for x in v], C.byref(r))
        return dict(solves=v[0].value, iters=v[1].value, fails=v[2].value, max_relres=r.value)

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.arpack_hip_dgen_destroy(self.h)
                self.h = None
        except Exception:
            pass

class ZGen:
    """Device operator pair of znaupd's generalized modes (bmat = 'G'; modes 2
    and 3, arpack_hip_zgen_create): mode 2 OP = inv[M] A, mode 3 OP = inv[A -
    sigma M] M with a complex sigma, B = M.  The inverse is the device BiCGStab
    to relative residual rtol on C = A - sigma M (mode 2: on M); ZRci.aupd_gen
    runs the whole loop with it."""

    def __init__(self, A: "ZCSR", M: "ZCSR", mode: int, sigma=0j, rtol: float = 1e-12,
                 maxit: int = 5000, method: str = "bicgstab"):
        L = lib()
        L.arpack_hip_zgen_create.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_int,
                                             C.c_double, C.c_double, C.c_double, C.c_int]
        L.arpack_hip_zgen_destroy.argtypes = [C.c_void_p]
        sigma = complex(sigma)
        h = C.c_void_p()
        rc = L.arpack_hip_zgen_create(C.byref(h), A.h, M.h, int(mode), sigma.real, sigma.imag,
                                      float(rtol), int(maxit))
        if rc != 0:
            raise RuntimeError(f"arpack_hip_zgen_create failed ({rc})")
        self.h, self.A, self.M, self.mode, self.sigma = h, A, M, int(mode), sigma
        if method != "bicgstab":  # "tridiag": A and M tridiagonal, a direct solve of C
            L.arpack_hip_zgen_set_method.argtypes = [C.c_void_p, C.c_int]
            if L.arpack_hip_zgen_set_method(self.h, {"tridiag": 1}[method]) != 0:
                raise ValueError(method)

    def stats(self):
        L = lib()
        L.arpack_hip_zgen_stats.argtypes = [C.c_void_p] + [C.POINTER(C.c_longlong)] * 3 + [_PD]
        v = [C.c_longlong() for _ in range(3)]
        r = C.c_double()
        L.arpack_hip_zgen_stats(self.h, *[C.byref(x) for x in v], C.byref(r))
        return dict(solves=v[0].value, iters=v[1].value, fails=v[2].value, max_relres=r.value)

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.arpack_hip_zgen_destroy(self.h)
                self.h = None
        except Exception:
            pass


class ZRci:
    """znaupd/zneupd state (SRC/znaupd.f, SRC/zneupd.f): complex128 arrays,
    ipntr(14), lworkl = 3*ncv^2 + 5*ncv, rwork(ncv).  Host arrays; the caller
    applies OP on workd slices (ido = -1/1; B*x at ipntr(3) in mode 3)."""

    def __init__(self, n, nev, ncv, which="LM", tol=0.0, bmat="I", mode=1, mxiter=300, ishift=1,
                 v0=None, prec="z"):
        """prec="c": the complex64 family (cnaupd / cneupd)."""
        self.n, self.nev, self.ncv = n, nev, ncv
        self.which, self.bmat, self.tol, self.mode = which, bmat, float(tol), mode
        self.prec = prec
        self.ct = np.complex64 if prec == "c" else np.complex128
        self.ido = np.zeros(1, np.int32)
        self.info = np.zeros(1, np.int32)
        self.iparam = np.zeros(11, np.int32)
        self.ipntr = np.zeros(14, np.int32)
        self.iparam[0], self.iparam[2], self.iparam[6] = ishift, mxiter, mode
        self.lworkl = 3 * ncv * ncv + 5 * ncv
        self.workl = np.zeros(self.lworkl, self.ct)
        self.rwork = np.zeros(ncv, np.float32 if prec == "c" else np.float64)
        self.resid = np.zeros(n, self.ct) if v0 is None else np.array(v0, self.ct)
        self.v = np.zeros(ncv * n, self.ct)
        self.workd = np.zeros(3 * n, self.ct)
        self.info[0] = 0 if v0 is None else 1

    def aupd(self):
        """One znaupd_c / cnaupd_c call (tol by value, SRC/icbazn.F90); returns ido."""
        f = getattr(lib(), self.prec + "naupd_c")
        f.argtypes = [_PI, C.c_char_p, _I, C.c_char_p, _I,
                      C.c_float if self.prec == "c" else C.c_double, _PD, _I, _PD, _I, _PI, _PI,
                      _PD, _PD, _I, _PD, _PI]
        f(_ip(self.ido), self.bmat.encode(), self.n, self.which.encode(), self.nev, self.tol,
          self.resid.ctypes.data, self.ncv, self.v.ctypes.data, self.n, _ip(self.iparam),
          _ip(self.ipntr), self.workd.ctypes.data, self.workl.ctypes.data, self.lworkl,
          self.rwork.ctypes.data, _ip(self.info))
        return int(self.ido[0])

    def aupd_zcsr(self, A: "ZCSR"):
        """Whole loop on the GPU with OP = A (mode 1)."""
        tol = C.c_double(self.tol)
        lib().arpack_hip_znaupd_zcsr(A.h, _ip(self.ido), self.bmat.encode(), self.n,
                                     self.which.encode(), self.nev, C.byref(tol),
                                     self.resid.ctypes.data, self.ncv, self.v.ctypes.data, self.n,
                                     _ip(self.iparam), _ip(self.ipntr), self.workd.ctypes.data,
                                     self.workl.ctypes.data, self.lworkl, self.rwork.ctypes.data,
                                     _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def aupd_zshift(self, S: "ZShift"):
        """Whole loop on the GPU in mode 3 (construct with mode=3): OP =
        (A - sigma I)^{-1} by the device solve S (arpack_hip_znaupd_zshift)."""
        tol = C.c_double(self.tol)
        lib().arpack_hip_znaupd_zshift(S.h, _ip(self.ido), self.bmat.encode(), self.n,
                                       self.which.encode(), self.nev, C.byref(tol),
                                       self.resid.ctypes.data, self.ncv, self.v.ctypes.data,
                                       self.n, _ip(self.iparam), _ip(self.ipntr),
                                       self.workd.ctypes.data, self.workl.ctypes.data,
                                       self.lworkl, self.rwork.ctypes.data, _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def aupd_gen(self, G: "ZGen"):
        """Whole loop on the GPU in znaupd's generalized modes (construct with
        bmat="G" and G's mode): OP*x and B*x by the device operator pair G
        (arpack_hip_znaupd_gen)."""
        tol = C.c_double(self.tol)
        L = lib()
        L.arpack_hip_znaupd_gen.argtypes = L.arpack_hip_znaupd_zshift.argtypes
        L.arpack_hip_znaupd_gen(G.h, _ip(self.ido), self.bmat.encode(), self.n,
                                self.which.encode(), self.nev, C.byref(tol),
                                self.resid.ctypes.data, self.ncv, self.v.ctypes.data, self.n,
                                _ip(self.iparam), _ip(self.ipntr), self.workd.ctypes.data,
                                self.workl.ctypes.data, self.lworkl, self.rwork.ctypes.data,
                                _ip(self.info))
        self.tol = tol.value
        return int(self.ido[0])

    def slice(self, k):
        o = int(self.ipntr[k]) - 1
        return self.workd[o:o + self.n]

    def eupd(self, rvec=True, howmny="A", sigma=0j, z=None):
        """zneupd_c: returns (d, Z (n x nconv), nconv); `z` may be self.v (Z = V,
        as the reference's drivers call it)."""
        nconv = int(self.iparam[4])
        d = np.zeros(self.nev + 1, self.ct)
        if z is None:
            z = np.zeros((self.nev + 1) * self.n, self.ct)
        select = np.zeros(self.ncv, np.int32)
        workev = np.zeros(2 * self.ncv, self.ct)
        info = np.zeros(1, np.int32)
        f = getattr(lib(), self.prec + "neupd_c")
        cs = _CF if self.prec == "c" else _CD
        f.argtypes = [_I, C.c_char_p, _PI, _PD, _PD, _I, cs, _PD, C.c_char_p, _I, C.c_char_p, _I,
                      C.c_float if self.prec == "c" else C.c_double, _PD, _I, _PD, _I, _PI, _PI,
                      _PD, _PD, _I, _PD, _PI]
        f(1 if rvec else 0, howmny.encode(), _ip(select), d.ctypes.data, z.ctypes.data, self.n,
          cs(sigma.real, sigma.imag), workev.ctypes.data, self.bmat.encode(), self.n,
          self.which.encode(), self.nev, self.tol, self.resid.ctypes.data, self.ncv,
          self.v.ctypes.data, self.n, _ip(self.iparam), _ip(self.ipntr), self.workd.ctypes.data,
          self.workl.ctypes.data, self.lworkl, self.rwork.ctypes.data, _ip(info))
        if info[0] < 0:
            raise ArpackError("zneupd", int(info[0]))
        return d[:nconv], z[:nconv * self.n].reshape(nconv, self.n).T, nconv

    @property
    def ritz(self):
        o = int(self.ipntr[5]) - 1
        return self.workl[o:o + self.ncv].copy()


class _CD(C.Structure):
    """C99 double _Complex passed by value (two doubles in SSE registers)."""
    _fields_ = [("re", C.c_double), ("im", C.c_double)]


class _CF(C.Structure):
    """C99 float _Complex passed by value (both floats in one SSE register)."""
    _fields_ = [("re", C.c_float), ("im", C.c_float)]


def eigsh(op, n, nev=6, ncv=None, which="LM", tol=0.0, v0=None, mxiter=300, rvec=True,
          device=False, sigma=None, rtol=1e-12, maxit=1000, solver="minres"):
    """Drive the RCI loop with a user OP (callable y = op(x) on workd slices), like
    TESTS/icb_arpack_c.c:60-65.  In device mode `op(x_addr, y_addr)` receives device
    addresses.  With `op` a CSR, the loop runs entirely on the GPU
    (arpack_hip_dsaupd_csr); with a CSR and `sigma`, in shift-invert mode 3 with
    OP = (A - sigma I)^{-1} by the device solve (DShift: `solver` "minres", any
    sigma, or "cg", cheaper, A - sigma I positive definite), the eigenvalues of A
    nearest sigma returned (dseupd's transform).
    Returns (d, Z, info-dict)."""
    ncv = ncv or min(n, max(2 * nev + 1, 20))
    if sigma is not None and not isinstance(op, CSR):
        raise ValueError("sigma needs a CSR operator (the device solve); with a callable, "
                         "drive SymRci(mode=3) and apply (A - sigma I)^{-1} yourself")
    shift = sigma is not None
    s = SymRci(n, nev, ncv, which, tol, mode=3 if shift else 1, mxiter=mxiter, v0=v0,
               device=device)
    if shift:
        S = DShift(op, sigma, rtol=rtol, maxit=maxit, method=solver)
        s.aupd_shift(S)
        if s.tol <= 0.0:
            s.tol = float(np.finfo(np.float64).eps / 2)
    elif isinstance(op, CSR):
        s.aupd_csr(op)
    else:
        while True:
            ido = s.aupd()
            if ido in (-1, 1):
                if device:
                    op(s.slice(0), s.slice(1))
                else:
                    s.slice(1)[:] = op(s.slice(0))
            elif ido == 99:
                break
            else:
                raise ArpackError("dsaupd", int(s.info[0]), {"ido": ido})
    if s.info[0] < 0:
        raise ArpackError("dsaupd", int(s.info[0]))
    res = dict(info=int(s.info[0]), iters=int(s.iparam[2]), nconv=int(s.iparam[4]),
               nopx=int(s.iparam[8]), nrorth=int(s.iparam[10]), ritz=s.ritz)
    d, z, nconv = s.eupd(rvec=rvec, sigma=float(sigma) if shift else 0.0)
    if rvec:
        if device:
            z = z.numpy().reshape(s.nev, n)[:nconv].T
        else:
            z = z.reshape(s.nev, n)[:nconv].T
    return d, (z if rvec else None), res


def _ns_vectors(dr, di, z, n, nconv):
    """dneupd's real Z (SRC/dneupd.f:81-91: a complex pair's eigenvector is
    z(:,j) +/- i z(:,j+1), the pair stored at dr(j) +/- i di(j)) -> complex columns."""
    Z = np.asarray(z).reshape(-1, n)[:nconv + 1].T
    out = np.zeros((n, nconv), np.complex128)
    j = 0
    while j < nconv:
        if di[j] != 0.0 and j + 1 < Z.shape[1]:
            v = Z[:, j] + 1j * Z[:, j + 1]
            out[:, j] = v
            if j + 1 < nconv:
                out[:, j + 1] = np.conj(v)
            j += 2
        else:
            out[:, j] = Z[:, j]
            j += 1
    return out


def eigs(op, n, nev=6, ncv=None, which="LM", tol=0.0, v0=None, mxiter=300, rvec=True,
         sigma=None, rtol=1e-12, maxit=200):
    """Nonsymmetric / complex counterpart of eigsh (the calling pattern of
    EXAMPLES/NONSYM/dndrv1.f and EXAMPLES/COMPLEX/zndrv1.f / zndrv2.f):

      * op a CSR: dnaupd with OP = A on the GPU (arpack_hip_dnaupd_csr_cycles);
      * op a ZCSR: znaupd with OP = A on the GPU, or with sigma given, shift-invert
        mode 3 with OP = (A - sigma I)^{-1} by the device BiCGStab (ZShift, to
        rtol within maxit iterations) -- eigenvalues of A returned (zneupd's
        transform);
      * op a CSR and a real sigma: dnaupd in shift-invert mode 3 with OP =
        (A - sigma I)^{-1} by the device BiCGStab (DShift);
      * op a callable y = op(x) on host vectors: the dnaupd RCI loop (real x).

    Returns (d, Z, info-dict) with complex eigenvalues d (nconv of them) and,
    if rvec, complex eigenvectors as the columns of Z."""
    ncv = ncv or min(n, max(2 * nev + 1, 20))
    if isinstance(op, ZCSR):
        mode = 1 if sigma is None else 3
        s = ZRci(n, nev, ncv, which, tol, mode=mode, mxiter=mxiter, v0=v0)
        if sigma is None:
            s.aupd_zcsr(op)
        else:
            S = ZShift(op, sigma, rtol=rtol, maxit=maxit)
            s.aupd_zshift(S)
        if s.info[0] < 0:
            raise ArpackError("znaupd", int(s.info[0]))
        res = dict(info=int(s.info[0]), iters=int(s.iparam[2]), nconv=int(s.iparam[4]),
                   nopx=int(s.iparam[8]))
        d, z, nconv = s.eupd(rvec=rvec, sigma=0j if sigma is None else complex(sigma))
        return d, (z if rvec else None), res
    if sigma is not None and not isinstance(op, CSR):
        raise ValueError("sigma needs a CSR or ZCSR operator (the device solve); with a "
                         "callable, drive NsRci(mode=3) and apply (A - sigma I)^{-1} yourself")
    shift = sigma is not None
    s = NsRci(n, nev, ncv, which, tol, mode=3 if shift else 1, mxiter=mxiter, v0=v0)
    if shift:  # real shift-invert: OP = (A - sigma I)^{-1} by the device BiCGStab
        S = DShift(op, float(sigma), rtol=rtol, maxit=maxit, method="bicgstab")
        s.aupd_shift(S)
        if s.tol <= 0.0:
            s.tol = float(np.finfo(np.float64).eps / 2)
    elif isinstance(op, CSR):
        s.aupd_csr(op)
    else:
        while True:
            ido = s.aupd()
            if ido in (-1, 1):
                s.slice(1)[:] = op(s.slice(0))
            elif ido == 99:
                break
            else:
                raise ArpackError("dnaupd", int(s.info[0]), {"ido": ido})
    if s.info[0] < 0:
        raise ArpackError("dnaupd", int(s.info[0]))
    res = dict(info=int(s.info[0]), iters=int(s.iparam[2]), nconv=int(s.iparam[4]),
               nopx=int(s.iparam[8]))
    dr, di, z, nconv = s.eupd(rvec=rvec, sigmar=float(sigma) if shift else 0.0)
    d = dr + 1j * di
    return d, (_ns_vectors(dr, di, z, n, nconv) if rvec else None), res


# ----------------------------------------------------------- multi-GPU (RCCL)
def _declare_dist(L):
    L.arpack_hip_comm_unique_id.argtypes = [C.c_char_p]
    L.arpack_hip_comm_init.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_int]
    L.arpack_hip_comm_allreduce.argtypes = [C.c_void_p, C.c_int]
    L.arpack_hip_dist_create.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_int64, C.c_int64]
    L.arpack_hip_dist_destroy.argtypes = [C.c_void_p]
    L.arpack_hip_dist_info.argtypes = [C.c_void_p] + [C.POINTER(C.c_int64)] * 4
    L.arpack_hip_dist_rows.argtypes = [C.POINTER(C.c_void_p), C.c_int64, C.c_int64, C.c_int64]
    for f in (L.arpack_hip_pdsaupd_c, L.arpack_hip_pdnaupd_c):
        f.argtypes = [C.c_void_p, _PI, C.c_char_p, _I, C.c_char_p, _I, C.c_double, _PD, _I, _PD,
                      _I, _PI, _PI, _PD, _PD, _I, _PI]
        f.restype = None
    L.arpack_hip_pdseupd_c.argtypes = [C.c_void_p] + L.dseupd_c.argtypes
    L.arpack_hip_pdneupd_c.argtypes = [C.c_void_p] + L.dneupd_c.argtypes
    L.arpack_hip_pdsaupd_csr_cycles.argtypes = [C.c_void_p, _I, _PI, C.c_char_p, _I, C.c_char_p,
                                                _I, C.POINTER(C.c_double), _PD, _I, _PD, _I, _PI,
                                                _PI, _PD, _PD, _I, _PI]
    L.arpack_hip_pdnaupd_csr_cycles.argtypes = L.arpack_hip_pdsaupd_csr_cycles.argtypes


def comm_unique_id() -> bytes:
    L = lib()
    _declare_dist(L)
    buf = C.create_string_buffer(128)
    if L.arpack_hip_comm_unique_id(buf) != 0:
        raise RuntimeError("ncclGetUniqueId failed")
    return buf.raw


def comm_init(nranks: int, rank: int, uid: bytes, device: int = 0):
    """Create the engine's RCCL communicator (one process per GPU)."""
    L = lib()
    _declare_dist(L)
    if L.arpack_hip_comm_init(nranks, rank, C.c_char_p(bytes(uid)), device) != 0:
        raise RuntimeError("ncclCommInitRank failed")


_HOST_ALLREDUCE = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_int, C.c_void_p)
_HOST_P2P = C.CFUNCTYPE(None, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                        C.POINTER(C.POINTER(C.c_double)), C.POINTER(C.c_int64), C.c_void_p)
_host_cbs = None


def comm_init_host(nranks: int, rank: int, device: int = 0):
    """Engine communicator over the host-staged transport: every allreduce and
    every point-to-point group of the distributed SpMV goes through
    torch.distributed (the default process group, e.g. gloo) instead of RCCL --
    for rehearsing several ranks where RCCL cannot run them (more ranks than
    GPUs).  The groups are the ones RCCL runs (same device slices, counts and
    offsets); only the wire differs.  arpack_hip_comm_init_host."""
    import torch
    import torch.distributed as dist
    global _host_cbs

    def allreduce(buf, count, ctx):
        a = np.ctypeslib.as_array(buf, (count,))
        t = torch.from_numpy(a.copy())
        dist.all_reduce(t)
        a[:] = t.numpy()

    def p2p(nops, peer, is_send, bufs, count, ctx):
        # every transfer posted non-blocking, then all completed (arpack_hip.h:
        # transfers between a pair match in posting order)
        reqs, recv = [], []
        for k in range(nops):
            cnt = int(count[k])
            a = np.ctypeslib.as_array(bufs[k], (cnt,))
            if is_send[k]:
                t = torch.from_numpy(a.copy())
                reqs.append((dist.isend(t, int(peer[k])), t))
            else:
                t = torch.empty(cnt, dtype=torch.float64)
                reqs.append((dist.irecv(t, int(peer[k])), t))
                recv.append((a, t))
        for q, _ in reqs:
            q.wait()
        for a, t in recv:
            a[:] = t.numpy()

    L = lib()
    _declare_dist(L)
    cbs = (_HOST_ALLREDUCE(allreduce), _HOST_P2P(p2p))
    L.arpack_hip_comm_init_host.argtypes = [C.c_int, C.c_int, _HOST_ALLREDUCE, _HOST_P2P,
                                            C.c_void_p, C.c_int]
    if L.arpack_hip_comm_init_host(nranks, rank, cbs[0], cbs[1], None, device) != 0:
        raise RuntimeError("arpack_hip_comm_init_host failed")
    _host_cbs = cbs  # the C side holds these function pointers


def comm_destroy():
    lib().arpack_hip_comm_destroy()


def comm_size() -> int:
    """Ranks of the engine's communicator (arpack_hip_comm_size; 1 without one)."""
    return lib().arpack_hip_comm_size()


def comm_failed() -> bool:
    """True once a collective of the engine's communicator failed
    (arpack_hip_comm_failed); the solves then end with info = -9999."""
    return lib().arpack_hip_comm_failed() != 0


def partition_rows(n: int, nranks: int, rank: int):
    """Contiguous balanced row blocks (PARPACK/TESTS/MPI/icb_parpack_c.c:60-77)."""
    base, rem = divmod(n, nranks)
    r0 = rank * base + min(rank, rem)
    return r0, r0 + base + (1 if rank < rem else 0)


class DistOp:
    """This rank's rows of a row-block distributed operator (collective setup)."""

    def __init__(self, A: CSR, n_global: int, row0: int):
        L = lib()
        _declare_dist(L)
        h = C.c_void_p()
        rc = L.arpack_hip_dist_create(C.byref(h), A.h, n_global, row0)
        if rc != 0:
            raise RuntimeError(f"arpack_hip_dist_create failed ({rc})")
        self.h = h
        self.A = A  # keeps the local CSR alive
        self.n_global, self.row0, self.nloc = n_global, row0, A.n

    def matvec_device(self, x, y):
        """y = A x on this rank's rows (collective; DeviceBuffers or addresses)."""
        xp = x if isinstance(x, int) else _ptr(x)
        yp = y if isinstance(y, int) else _ptr(y)
        L = lib()
        L.arpack_hip_dist_spmv.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        if L.arpack_hip_dist_spmv(self.h, xp, yp) != 0:
            raise RuntimeError("distributed spmv failed")

    def info(self):
        v = [C.c_int64() for _ in range(4)]
        lib().arpack_hip_dist_info(self.h, *[C.byref(x) for x in v])
        return dict(zip(["halo_lo", "halo_hi", "send_lo", "send_hi"], [x.value for x in v]))

    @property
    def mode(self):
        """Exchange form: "halo" (neighbour slabs), "ghosts" (per-peer ghost
        lists) or "allgather" (arpack_hip_dist_mode)."""
        L = lib()
        L.arpack_hip_dist_mode.argtypes = [C.c_void_p]
        return ("halo", "ghosts", "allgather")[L.arpack_hip_dist_mode(self.h)]

    @property
    def spill(self):
        """True when the symmetric-storage SpMV sends a forward spill
        (arpack_hip_dist_spill); False for full storage or the spill-free form."""
        L = lib()
        L.arpack_hip_dist_spill.argtypes = [C.c_void_p]
        return L.arpack_hip_dist_spill(self.h) == 1

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.arpack_hip_dist_destroy(self.h)
                self.h = None
        except Exception:
            pass


class DistRows:
    """This rank's row block [row0, row0 + nloc) of an n_global-row problem with
    no operator attached: the PARPACK RCI use, where the caller applies OP to its
    local rows (arpack_hip_dist_rows)."""

    def __init__(self, nloc: int, row0: int, n_global: int):
        L = lib()
        _declare_dist(L)
        h = C.c_void_p()
        rc = L.arpack_hip_dist_rows(C.byref(h), nloc, row0, n_global)
        if rc != 0:
            raise RuntimeError(f"arpack_hip_dist_rows failed ({rc})")
        self.h = h
        self.n_global, self.row0, self.nloc = n_global, row0, nloc

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.arpack_hip_dist_destroy(self.h)
                self.h = None
        except Exception:
            pass


def pxaupd(s, D: DistRows) -> int:
    """One collective pdsaupd_c / pdnaupd_c call (ICB/parpack.h:17-33) on this
    rank's slice: s is a SymRci or NsRci built with n = local rows."""
    f = lib().arpack_hip_pdnaupd_c if isinstance(s, NsRci) else lib().arpack_hip_pdsaupd_c
    f(D.h, _ip(s.ido), s.bmat.encode(), s.n, s.which.encode(), s.nev, s.tol, _ptr(s.resid),
      s.ncv, _ptr(s.v), s.ldv, _ip(s.iparam), _ip(s.ipntr), _ptr(s.workd), s.workl.ctypes.data,
      s.lworkl, _ip(s.info))
    return int(s.ido[0])


def pdsaupd_cycles(s: "SymRci", D: DistOp, max_cycles: int) -> int:
    """Distributed free-running dsaupd (dnaupd for an NsRci) on this rank's
    slice (s.n = local rows)."""
    tol = C.c_double(s.tol)
    f = (lib().arpack_hip_pdnaupd_csr_cycles if isinstance(s, NsRci)
         else lib().arpack_hip_pdsaupd_csr_cycles)
    f(D.h, int(max_cycles), _ip(s.ido), s.bmat.encode(), s.n, s.which.encode(), s.nev,
      C.byref(tol), _ptr(s.resid), s.ncv, _ptr(s.v), s.ldv, _ip(s.iparam), _ip(s.ipntr),
      _ptr(s.workd), s.workl.ctypes.data, s.lworkl, _ip(s.info))
    s.tol = tol.value
    return int(s.ido[0])
