#!/bin/bash
# Round 6, box 18: znaupd's generalized modes with the direct tridiagonal
# solve of C (zndrv3/zndrv4.f's zgttrf), beside BiCGStab.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06r \
  "zgen|300|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_zgen.py"
