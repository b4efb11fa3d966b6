#!/bin/bash
# Round 6, box 20: the whole GPU suite and smoke on the final tree.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06u \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|1000|python -u -m pytest -v --durations=20 --timeout 300 --timeout-method thread -m gpu tests"
