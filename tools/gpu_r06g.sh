#!/bin/bash
# Round 6, box 7: the device tridiagonal direct solve (m7, m8/m9), and the
# dshift / generalized / modes suites around it.
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06g \
  "tri|600|$T tests/test_gpu_dshift.py tests/test_gpu_gen.py tests/test_gpu_modes.py"
