"""Record the expected output of the reference's own test programs.

oracle/Makefile (target `reftests`) compiles arpack-ng's TESTS/*.f where they
lie under /root/reference and links each twice: <t>_ref against the reference
built from its own sources (oracle/_ref/libarpack_ref.so) and <t>_hip against
libarpack_hip.so. This script runs the *_ref programs here (CPU) and stores
their stdout and exit status as fixtures under tests/golden/reftests/ (the
example drivers of EXAMPLES/ as ex_<driver>.out);
tests/test_gpu_reftests.py runs the *_hip programs on the GPU and compares.
testA.mtx is the data file TESTS/dnsimp.f reads (the reference's own fixture).

    make -C oracle reftests && python tests/golden/make_reftests.py
"""
import json
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.path.join(ROOT, "oracle", "_ref", "tests")
OUT = os.path.join(ROOT, "tests", "golden", "reftests")
TESTS = ["bug_142", "bug_142_gen", "bug_58_double", "bug_1323", "bug_79_double_complex", "dnsimp"]
# the example drivers (EXAMPLES/*/), built as oracle/_ref/tests/ex_<driver>_{ref,hip}
EXAMPLES = sorted(f[3:-4] for f in os.listdir(BIN) if f.startswith("ex_") and f.endswith("_ref")) \
    if os.path.isdir(BIN) else []


def main():
    os.makedirs(OUT, exist_ok=True)
    rcs = {}
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(os.path.join(OUT, "testA.mtx"), d)
        for t in TESTS + ["ex_" + e for e in EXAMPLES]:
            r = subprocess.run([os.path.join(BIN, t + "_ref")], cwd=d, capture_output=True,
                               text=True, timeout=120)
            rcs[t] = r.returncode
            with open(os.path.join(OUT, t + ".out"), "w") as f:
                f.write(r.stdout)
            print(t, "rc", r.returncode)
    with open(os.path.join(OUT, "rc.json"), "w") as f:
        json.dump(rcs, f, indent=1)


if __name__ == "__main__":
    main()
