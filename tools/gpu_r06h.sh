#!/bin/bash
# Round 6, box 8: znaupd's generalized modes on the device, then the whole GPU
# suite on the round-6 tree (slowest tests listed).
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06h \
  "zgen|240|$T tests/test_gpu_zgen.py" \
  "suite|1000|python -u -m pytest -v --durations=30 --timeout 300 --timeout-method thread -m gpu tests"
