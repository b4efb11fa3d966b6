#!/bin/bash
# Round 6, box 19: dnaupd's complex shifts on the device (dndrv5/6.f), and the
# generalized-mode suites around them.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06s \
  "gen|400|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gen.py tests/test_gpu_modes.py"
