#!/bin/bash
# Round 6, box 8: the whole GPU suite on the round-6 tree (slowest tests listed).
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06h \
  "suite|1080|python -u -m pytest -v --durations=30 --timeout 300 --timeout-method thread -m gpu tests"
