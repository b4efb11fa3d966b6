#!/bin/bash
# Round 6, box 17: the complex direct tridiagonal solve (ztri.hip) and
# zndrv2's shift-invert run with it.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06q \
  "zshift|300|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_zshift.py"
