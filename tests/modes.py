"""Caller-side operators for the spectral-transformation modes (the user half of
the RCI contract, EXAMPLES/SYM/dsdrv2-6.f and EXAMPLES/NONSYM/dndrv2-3.f):
1-D finite-element stiffness/mass pairs and the OP/B applications each mode asks
for at ido = -1 / 1 / 2.  Shared by tests/golden/make_golden.py (driving the
reference) and tests/test_gpu_modes.py (driving the engine) so both see the
same caller."""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spl


def fem1d(n):
    """A = (1/h) tridiag(-1, 2, -1), M = (h/6) tridiag(1, 4, 1), h = 1/(n+1)
    (the stiffness/mass pair of EXAMPLES/SYM/dsdrv3.f)."""
    h = 1.0 / (n + 1)
    e = np.ones(n)
    A = sp.diags([-e[1:], 2 * e, -e[1:]], [-1, 0, 1], format="csc") / h
    Mm = sp.diags([e[1:], 4 * e, e[1:]], [-1, 0, 1], format="csc") * (h / 6.0)
    return A, Mm


def convdiff1d(n, rho):
    """EXAMPLES/NONSYM/dndrv2.f / dndrv3.f operator: -u'' + rho u' on (0,1)."""
    h = 1.0 / (n + 1)
    e = np.ones(n)
    s = rho / 2.0
    A = sp.diags([(-1.0 / h - s) * e[1:], (2.0 / h) * e, (-1.0 / h + s) * e[1:]], [-1, 0, 1],
                 format="csc")
    Mm = sp.diags([e[1:], 4 * e, e[1:]], [-1, 0, 1], format="csc") * (h / 6.0)
    return A, Mm


class Caller:
    """op(x, ido, bx) and bop(x) for one (problem, mode, sigma).  For mode 2
    the RCI contract also wants A*x written back over x: exposed as `.ax`
    (EXAMPLES/SYM/dsdrv3.f:299-302)."""

    def __init__(self, kind, mode, n, sigma=0.0, rho=10.0):
        self.mode, self.sigma = mode, sigma
        A, Mm = fem1d(n) if kind == "fem1d" else convdiff1d(n, rho)
        self.A, self.M = A, Mm
        self.bmat = "I"
        self.ax = None
        if mode == 1:
            self.op = lambda x, ido=None, bx=None: A @ x
        elif mode == 2:  # generalized, OP = inv(M) A, B = M
            self.bmat = "G"
            lu = spl.splu(Mm)

            def op(x, ido=None, bx=None):
                self.ax = A @ x
                return lu.solve(self.ax)
            self.op = op
        elif mode == 3:  # shift-invert, OP = inv(A - sigma M) M, B = M
            self.bmat = "G"
            lu = spl.splu((A - sigma * Mm).tocsc())
            self.op = lambda x, ido=None, bx=None: lu.solve(Mm @ x if bx is None or ido == -1
                                                            else bx)
        elif mode == 4:  # buckling, OP = inv(K - sigma KG) K, B = K (K = A, KG = M)
            self.bmat = "G"
            lu = spl.splu((A - sigma * Mm).tocsc())
            self.op = lambda x, ido=None, bx=None: lu.solve(A @ x if bx is None or ido == -1
                                                            else bx)
        elif mode == 5:  # Cayley, OP = inv(A - sigma M)(A + sigma M), B = M
            self.bmat = "G"
            lu = spl.splu((A - sigma * Mm).tocsc())
            self.op = lambda x, ido=None, bx=None: lu.solve(
                A @ x + sigma * (Mm @ x if bx is None or ido == -1 else bx))
        self.bop = (lambda x: A @ x) if mode == 4 else (lambda x: Mm @ x)


def zconvdiff1d(n, rho):
    """EXAMPLES/COMPLEX/zndrv3.f / zndrv4.f operator pair: -u'' + rho u' on (0,1)
    with a complex rho, M = (h/6) tridiag(1, 4, 1), both complex128."""
    h = 1.0 / (n + 1)
    e = np.ones(n, np.complex128)
    s = complex(rho) / 2.0
    A = sp.diags([(-1.0 / h - s) * e[1:], (2.0 / h) * e, (-1.0 / h + s) * e[1:]], [-1, 0, 1],
                 format="csc", dtype=np.complex128)
    Mm = sp.diags([e[1:], 4 * e, e[1:]], [-1, 0, 1], format="csc", dtype=np.complex128) * (h / 6.0)
    return A, Mm


class ZCaller:
    """znaupd's generalized modes (bmat = 'G'; SRC/znaupd.f:23-31): mode 2 OP =
    inv(M) A, mode 3 OP = inv(A - sigma M) M (M x handed over at ido = 1),
    B = M -- the caller loops of zndrv3.f / zndrv4.f with a sparse LU."""

    def __init__(self, mode, n, sigma=0j, rho=10.0):
        self.mode, self.sigma, self.bmat = mode, complex(sigma), "G"
        A, Mm = zconvdiff1d(n, rho)
        self.A, self.M = A, Mm
        if mode == 2:
            lu = spl.splu(Mm.tocsc())
            self.op = lambda x, ido=None, bx=None: lu.solve(A @ x)
        else:
            lu = spl.splu((A - self.sigma * Mm).tocsc())
            self.op = lambda x, ido=None, bx=None: lu.solve(Mm @ x if bx is None or ido == -1
                                                            else bx)
        self.bop = lambda x: Mm @ x


def dndrv5_pair(n):
    """EXAMPLES/NONSYM/dndrv5.f / dndrv6.f pair: A = tridiag(-2, 2, 3),
    M = tridiag(1, 4, 1)."""
    e = np.ones(n)
    A = sp.diags([-2.0 * e[1:], 2.0 * e, 3.0 * e[1:]], [-1, 0, 1], format="csc")
    Mm = sp.diags([e[1:], 4.0 * e, e[1:]], [-1, 0, 1], format="csc")
    return A, Mm


class CShiftCaller:
    """dnaupd's complex-shift modes (SRC/dnaupd.f:28-33): mode 3 OP =
    Re{inv[A - sigma M] M}, mode 4 OP = Im{...}, B = M -- the caller loops of
    dndrv5.f (real part) / dndrv6.f (imaginary part), the complex LU by SciPy."""

    def __init__(self, mode, n, sigma):
        self.mode, self.sigma, self.bmat = mode, complex(sigma), "G"
        A, Mm = dndrv5_pair(n)
        self.A, self.M = A, Mm
        lu = spl.splu((A.astype(np.complex128) - self.sigma * Mm).tocsc())
        part = np.real if mode == 3 else np.imag
        self.op = lambda x, ido=None, bx=None: part(lu.solve((Mm @ x if bx is None or ido == -1
                                                              else bx).astype(np.complex128)))
        self.bop = lambda x: Mm @ x
        self.ax = None


class StdShiftInvert:
    """Standard shift-invert, bmat = 'I': OP = inv(A - sigma I) (dsdrv2 / dndrv2)."""

    def __init__(self, kind, n, sigma, rho=10.0):
        A, _ = fem1d(n) if kind == "fem1d" else convdiff1d(n, rho)
        self.A, self.sigma, self.bmat, self.mode = A, sigma, "I", 3
        lu = spl.splu((A - sigma * sp.identity(n, format="csc")).tocsc())
        self.op = lambda x, ido=None, bx=None: lu.solve(x)
        self.bop = None
        self.ax = None
