"""CPU: the Python drivers' argument handling (arpack-ng_amd/__init__.py) that
needs no device: shift-invert asks for a device operator, and the eigenvector
assembly of dneupd's real Z (SRC/dneupd.f:81-91: a complex pair's eigenvector is
z(:,j) +/- i z(:,j+1)) is checked on a constructed Z."""
import numpy as np
import pytest


def test_sigma_needs_a_device_operator(pkg):
    for f in (pkg.eigsh, pkg.eigs):
        with pytest.raises(ValueError):
            f(lambda x: x, 10, 2, sigma=1.0)


def test_ns_vectors_pairs(pkg):
    n = 5
    rng = np.random.default_rng(0)
    Z = rng.standard_normal((4, n))   # columns of dneupd's Z, stored column-major
    dr = np.array([1.0, 2.0, 2.0, 3.0])
    di = np.array([0.0, 0.5, -0.5, 0.0])
    out = pkg._ns_vectors(dr, di, Z.ravel(), n, 4)
    np.testing.assert_array_equal(out[:, 0], Z[0])
    np.testing.assert_array_equal(out[:, 1], Z[1] + 1j * Z[2])
    np.testing.assert_array_equal(out[:, 2], Z[1] - 1j * Z[2])
    np.testing.assert_array_equal(out[:, 3], Z[3])
