"""GPU: the PARPACK-style RCI entries (arpack_hip_pdsaupd_c / pdnaupd_c,
ICB/parpack.h:17-33) on a one-rank RCCL communicator give bit-identical
results to the single-GPU dsaupd_c / dnaupd_ RCI on the same caller loop --
every reduction goes through the distributed finalize (partial sums ->
ncclAllReduce -> phase logic), so this pins the collective path of the user-OP
(PARPACK/EXAMPLES/MPI/pdsdrv1.f) use.  Multi-rank partitions of the same loop
are the driver's 8-GPU job; their host logic is covered by test_dist_plan.py."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
import modes  # noqa: E402
from oracle import matrices as M  # noqa: E402

pytestmark = pytest.mark.gpu


def _loop(s, step, op, bop=None, mode=1):
    while True:
        ido = step()
        if ido in (-1, 1):
            bx = s.slice(2).copy() if (mode >= 3 and ido == 1) else None
            s.slice(1)[:] = op(s.slice(0).copy(), ido, bx)
        elif ido == 2:
            s.slice(1)[:] = bop(s.slice(0).copy())
        elif ido == 99:
            return
        else:
            raise AssertionError(ido)


def _same(a, b):
    assert int(a.info[0]) == int(b.info[0]) == 0
    assert np.array_equal(a.iparam, b.iparam)
    assert np.array_equal(a.ipntr, b.ipntr)
    assert np.array_equal(a.workl, b.workl)
    assert np.array_equal(a.resid, b.resid)
    assert np.array_equal(a.v, b.v)


@pytest.fixture
def comm1(pkg):
    pkg.comm_init(1, 0, pkg.comm_unique_id(), 0)
    yield
    pkg.comm_destroy()


def test_pdsaupd_c_matches_dsaupd_c(pkg, golden, comm1):
    g = golden("g2_icb_ds")
    rp, col, val = M.diag(int(g["spec"][1]))
    A = M.to_scipy(rp, col, val)
    n, nev, ncv, tol = A.shape[0], int(g["nev"]), int(g["ncv"]), float(g["tol"])
    mk = lambda: pkg.SymRci(n, nev, ncv, str(g["which"]), tol, v0=g["v0"],  # noqa: E731
                            mxiter=int(g["mxiter"]), icb=True)
    op = lambda x, ido, bx: A @ x  # noqa: E731
    s1 = mk()
    _loop(s1, s1.aupd, op)
    D = pkg.DistRows(n, 0, n)
    s2 = mk()
    _loop(s2, lambda: pkg.pxaupd(s2, D), op)
    _same(s1, s2)
    assert int(s1.iparam[2]) == int(g["iparam"][2])
    d, _, nconv = s2.eupd(dist=D)
    np.testing.assert_allclose(np.sort(d), np.sort(g["d"]), rtol=1e-9)


def test_pdsaupd_c_generalized_mode3(pkg, golden, comm1):
    """bmat = 'G' (B-norms through the collective): dsdrv4-style shift-invert."""
    g = golden("m4_sym_gen_si")
    c = modes.Caller(str(g["kind"]), int(g["mode"]), int(g["n"]), float(g["sigma"]))
    n = int(g["n"])
    mk = lambda: pkg.SymRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]),  # noqa: E731
                            float(g["tol"]), bmat=c.bmat, mode=c.mode, mxiter=300, v0=g["v0"],
                            icb=True)
    s1 = mk()
    _loop(s1, s1.aupd, c.op, c.bop, c.mode)
    D = pkg.DistRows(n, 0, n)
    s2 = mk()
    _loop(s2, lambda: pkg.pxaupd(s2, D), c.op, c.bop, c.mode)
    _same(s1, s2)
    assert int(s2.iparam[2]) == int(g["iparam"][2])
    d1, z1, _ = s1.eupd(sigma=float(g["sigma"]))
    d2, z2, _ = s2.eupd(sigma=float(g["sigma"]), dist=D)
    assert np.array_equal(d1, d2) and np.array_equal(z1, z2)


def test_pdnaupd_c_matches_dnaupd(pkg, golden, comm1):
    g = golden("n2_dnsimp_tol")
    spec = g["spec"]
    rp, col, val = M.convdiff2d(int(spec[1]), float(spec[2]))
    A = M.to_scipy(rp, col, val)
    n = A.shape[0]
    mk = lambda: pkg.NsRci(n, int(g["nev"]), int(g["ncv"]), str(g["which"]),  # noqa: E731
                           float(g["tol"]), mxiter=int(g["mxiter"]), v0=g["v0"])
    op = lambda x, ido, bx: A @ x  # noqa: E731
    s1 = mk()
    _loop(s1, s1.aupd, op)
    D = pkg.DistRows(n, 0, n)
    s2 = mk()
    _loop(s2, lambda: pkg.pxaupd(s2, D), op)
    _same(s1, s2)
    assert int(s2.iparam[2]) == int(g["iparam"][2])
    r1, r2 = s1.eupd(), s2.eupd(dist=D)
    assert all(np.array_equal(a, b) for a, b in zip(r1, r2))


def test_overlapped_distributed_spmv_same_solve(tmp_path):
    """AHIP_DIST_OVERLAP=1 (opt-in): the distributed free run with the next
    step's halo + SpMV on a second stream and a split p2p communicator must
    give the same solve as the serialised schedule -- on a 1-rank RCCL
    communicator (bench.py --force-dist), the time-to-converge solve's restart
    cycles, OP*x count and converged count are equal with and without it.  Run
    in subprocesses: the switch is read once per process."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for ov in ("0", "1"):
        env = dict(os.environ, AHIP_DIST_OVERLAP=ov)
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--force-dist",
                            "--rows", "400000", "--steps", "3", "--warmup", "1",
                            "--no-cpu-baseline", "--no-full-storage", "--steady-cycles", "0"],
                           env=env, capture_output=True, text=True, timeout=300, cwd=root)
        assert r.returncode == 0, r.stderr[-3000:]
        res[ov] = json.loads(r.stdout.strip().splitlines()[-1])["time_to_converge"]
    for k in ("iters", "nopx", "nconv", "info"):
        assert res["0"][k] == res["1"][k], (k, res)
