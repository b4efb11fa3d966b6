#!/bin/bash
# Round 6, box 32: the full GPU suite and smoke on the final tree (1,024-thread
# complex tiles with six entries a lane).
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06ag \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|1000|python -u -m pytest -v --durations=20 --timeout 300 --timeout-method thread -m gpu tests"
