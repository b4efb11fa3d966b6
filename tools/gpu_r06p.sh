#!/bin/bash
# Round 6, box 16: the folded complex step on a 3-eigenvalue operator (Krylov
# spaces that close: parks, give-ups, restarts inside folded cycles).
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06p \
  "zfold|300|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_zfold.py"
