"""GPU: the complex Arnoldi step's fused update above 32 columns.

Up to 40 basis columns (config 5's ncv) `zs_update` subtracts V h and sums the
next DGKS sweep's partials [V^H r ; r^H r] in the same pass over V
(csrc/zstep.hip step_update); before, steps with j > 32 ran the update and then
separate partial passes (step_dots over the stored r).  The two forms sum the
same terms in the same per-thread order into the same partial slots, so a
solve must come out bitwise identical with AHIP_ZFUSE_MAX=32 (the split form)
and the default (fused), and both must match the reference's znaupd
(SRC/znaitr.f:585-590,675-690) in restart cycles and Ritz values.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import matrices as M
from oracle import ref

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not ref.available(), reason="oracle/_ref")]


def _solve(pkg, A, n, nev, ncv, v0, fuse_max):
    old = os.environ.get("AHIP_ZFUSE_MAX")
    os.environ["AHIP_ZFUSE_MAX"] = str(fuse_max)
    try:
        s = pkg.ZRci(n, nev, ncv, "LM", 1e-10, mxiter=300, v0=v0)
        while True:
            ido = s.aupd()
            if ido in (-1, 1):
                s.slice(1)[:] = A @ s.slice(0)
            elif ido == 99:
                break
            else:
                raise AssertionError(ido)
        d, z, nconv = s.eupd(rvec=True)
        return int(s.info[0]), int(s.iparam[2]), int(s.iparam[8]), d[:nconv].copy(), \
            np.array(z[:, :nconv]), nconv
    finally:
        if old is None:
            os.environ.pop("AHIP_ZFUSE_MAX", None)
        else:
            os.environ["AHIP_ZFUSE_MAX"] = old


def test_znaupd_ncv40_fused_equals_split(pkg):
    # well-separated dominant spectrum (100 e^{-i/300} + small complex coupling):
    # the reference converges in 7 cycles, so the count is not rounding-driven
    # (config 5's operator clusters its spectrum near 100: ~100 cycles at this
    # size, where one-ulp differences move the count by a few)
    n, nev, ncv = 6000, 10, 40
    rng = np.random.default_rng(11)
    B = sp.random(n, n, density=8.0 / n, random_state=rng, format="csr")
    B.data = (np.round(B.data * 64.0) / 256.0) * (1.0 + 1.0j)
    A = (B + sp.diags(100.0 * np.exp(-np.arange(n) / 300.0) + 0.0j)).tocsr()
    v0 = M.dlarnv_uniform(2 * n)[0].view(np.complex128)
    fused = _solve(pkg, A, n, nev, ncv, v0, 40)
    split = _solve(pkg, A, n, nev, ncv, v0, 32)
    assert fused[:3] == split[:3]
    assert np.array_equal(fused[3], split[3])  # bitwise: same partials either way
    assert np.array_equal(fused[4], split[4])
    want = ref.znaupd_solve(lambda x, *_: A @ x, n, nev, ncv, "LM", 1e-10, v0=v0, rvec=False)
    info, iters, _, d, Z, nconv = fused
    assert info == want["info"]
    assert iters == int(want["iparam"][2])
    assert nconv == want["nconv"]
    got, exp = np.sort_complex(d), np.sort_complex(want["d"])
    assert np.all(np.abs(got - exp) <= 1e-9 * max(1.0, np.abs(exp).max())), (got, exp)
    r = np.linalg.norm(A @ Z - Z * d, axis=0)
    assert np.all(r <= 1e-8 * np.abs(d).max()), r
