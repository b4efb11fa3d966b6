"""Record the expected output of the reference's own PARPACK (MPI) programs.

oracle/Makefile (target `parpack`) compiles PARPACK/EXAMPLES/MPI/p*drv*.f and
PARPACK/TESTS/MPI/issue46.f where they lie under /root/reference and links each
twice: p_<t>_ref against the reference's PARPACK built from its own sources
(oracle/_ref/libparpack_ref.so, with the image's MPICH) and p_<t>_hip against
arpack-ng_amd/libparpack_hip.so.  This script runs the *_ref programs here
(CPU) under `mpiexec -n P` for P = 1 and 2 -- the reference's own test runs use
`mpirun -n 2` (PARPACK/EXAMPLES/MPI/Makefile.am) -- and stores stdout and exit
status under tests/golden/preftests/ (<t>.np<P>.out, rc.json);
tests/test_gpu_parpack.py runs the *_hip programs the same way on the GPU box.

    make -C oracle parpack && python tests/golden/make_preftests.py
"""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.path.join(ROOT, "oracle", "_ref", "tests")
OUT = os.path.join(ROOT, "tests", "golden", "preftests")
MPIEXEC = "/opt/conda/bin/mpiexec"
PROGRAMS = ["pdsdrv1", "pdndrv1", "pdndrv3", "pssdrv1", "psndrv1", "psndrv3", "pcndrv1",
            "pzndrv1", "issue46"]


def main():
    os.makedirs(OUT, exist_ok=True)
    rcs = {}
    for t in PROGRAMS:
        for np_ in (1, 2):
            r = subprocess.run([MPIEXEC, "-n", str(np_), os.path.join(BIN, "p_%s_ref" % t)],
                               capture_output=True, text=True, timeout=300)
            key = "%s.np%d" % (t, np_)
            rcs[key] = r.returncode
            with open(os.path.join(OUT, key + ".out"), "w") as f:
                f.write(r.stdout)
            print(key, "rc", r.returncode)
    with open(os.path.join(OUT, "rc.json"), "w") as f:
        json.dump(rcs, f, indent=1)


if __name__ == "__main__":
    main()
