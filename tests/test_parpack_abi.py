"""CPU: PARPACK's boundary library (arpack-ng_amd/libparpack_hip.so) exports
every entry point of include/parpack.h (ICB/parpack.h:17-33), their Fortran
twins (PARPACK/SRC/MPI/p*aupd.f, p*eupd.f) and the collective norms the
reference's drivers call (pdnorm2.f, pdznorm2.f, psnorm2.f, pscnorm2.f); and
those norms, run under `mpiexec -n 2` without any GPU work, equal the global
2-norm (the MAX-then-scaled-SUM reduction of PARPACK/SRC/MPI/pdnorm2.f)."""
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "arpack-ng_amd", "libparpack_hip.so")
MPIEXEC = "/opt/conda/bin/mpiexec"
MPIINC = "/opt/conda/include"
MPIDIR = os.path.join(ROOT, "oracle", "_ref", "mpi")


def _exports():
    if not os.path.exists(LIB):
        pytest.skip("libparpack_hip.so not built (needs MPI headers)")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


def test_parpack_header_symbols_exported():
    txt = open(os.path.join(ROOT, "include", "parpack.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    declared = set(re.findall(r"\b(p[sdcz][sn][ae]upd_c)\s*\(", txt))
    assert len(declared) == 12
    ex = _exports()
    for s in sorted(declared):
        assert s in ex and s[:-1] in ex, s  # C entry and the Fortran symbol p??aupd_
    for s in ("pdnorm2_", "pdznorm2_", "psnorm2_", "pscnorm2_"):
        assert s in ex, s


NORM_PROG = r"""
#include <math.h>
#include <stdio.h>
#include "parpack.h"
double pdnorm2_(MPI_Fint*, a_int*, const double*, a_int*);
double pdznorm2_(MPI_Fint*, a_int*, const double*, a_int*);
int main() {
    MPI_Init(NULL, NULL);
    int r; MPI_Comm_rank(MPI_COMM_WORLD, &r);
    MPI_Fint c = MPI_Comm_c2f(MPI_COMM_WORLD);
    double x[6]; a_int n = 6, inc = 1, n3 = 3;
    for (int i = 0; i < 6; ++i) x[i] = (r + 1) * 1e150 * (i + 1);  /* overflow-safe path */
    double a = pdnorm2_(&c, &n, x, &inc), b = pdznorm2_(&c, &n3, x, &inc);
    if (r == 0) printf("%.17g %.17g\n", a, b);
    MPI_Finalize();
    return 0;
}
"""


def test_pdnorm2_collective(tmp_path):
    if not (os.path.exists(MPIEXEC) and os.path.exists(os.path.join(MPIDIR, "libmpi.so.12"))):
        pytest.skip("no MPICH runtime / oracle/_ref/mpi (make -C oracle parpack)")
    _exports()
    src = tmp_path / "norm.c"
    src.write_text(NORM_PROG)
    exe = str(tmp_path / "norm")
    lib = os.path.dirname(LIB)
    r = subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), "-I", MPIINC, str(src),
                        "-o", exe, "-L", lib, "-l:libparpack_hip.so", "-l:libarpack_hip.so",
                        "-Wl,-rpath," + lib, os.path.join(MPIDIR, "libmpi.so.12"),
                        "-Wl,-rpath," + MPIDIR, "-Wl,-rpath-link," + MPIDIR, "-lm"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([MPIEXEC, "-n", "2", exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    a, b = (float(t) for t in r.stdout.split())
    x = np.concatenate([(k + 1) * 1e150 * np.arange(1, 7) for k in range(2)])
    assert abs(a - np.linalg.norm(x)) <= 1e-14 * np.linalg.norm(x)
    assert abs(b - np.linalg.norm(x)) <= 1e-14 * np.linalg.norm(x)  # 3 complex = 6 reals a rank


def test_parpack_reference_fixtures_parse():
    """The recorded outputs of the reference's PARPACK programs
    (tests/golden/preftests, tests/golden/make_preftests.py) hold a Ritz table
    and the converged / cycle / OP*x counts the GPU test compares, for 1 and 2
    ranks, and every recorded run exited 0."""
    import json
    from test_gpu_reftests import parse
    gold = os.path.join(ROOT, "tests", "golden", "preftests")
    rcs = json.load(open(os.path.join(gold, "rc.json")))
    assert len(rcs) == 18 and all(v == 0 for v in rcs.values())
    for key in rcs:
        rows, counts = parse(open(os.path.join(gold, key + ".out")).read())
        assert rows and counts["nconv"] and counts["iters"] and counts["nopx"], key

