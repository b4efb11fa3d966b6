"""CPU: the complex generalized-mode fixtures z5-z7 (made by the reference's
znaupd/zneupd, tests/golden/make_golden.py zmode_fixtures) against an
independent dense solve of the same pencil A x = lambda M x (scipy.linalg.eig):
mode 2 (OP = inv(M) A, LM) gives the nev eigenvalues of largest magnitude,
mode 3 (OP = inv(A - sigma M) M, LM) the nev nearest sigma."""
import os
import sys

import numpy as np
import pytest
import scipy.linalg as sla

sys.path.insert(0, os.path.dirname(__file__))
import modes  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", ["z5_zgen", "z6_zgen_si", "z7_zgen_si_complex"])
def test_fixture_matches_dense_pencil(name):
    g = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    mode, n, sigma, rho = int(g["mode"]), int(g["n"]), complex(g["sigma"]), complex(g["rho"])
    nev = int(g["nev"])
    A, Mm = modes.zconvdiff1d(n, rho)
    lam = sla.eig(A.toarray(), Mm.toarray(), right=False)
    key = np.abs(lam) if mode == 2 else 1.0 / np.abs(lam - sigma)
    want = lam[np.argsort(-key)[:nev]]
    d = g["d"]
    assert int(g["info"]) == 0 and len(d) == nev
    for x in want:
        assert np.abs(d - x).min() <= 1e-8 * np.abs(want).max(), (x, d)
