#!/bin/bash
# Round 6, box 26: config 5's profile set on the 1,024-thread complex tiles
# (kernel trace + FETCH_SIZE / WRITE_SIZE passes), then the full GPU suite and
# smoke on the final tree.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06aa \
  "prof_c5|600|bash tools/profile_c5.sh r06aa_c5" \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|1000|python -u -m pytest -v --durations=20 --timeout 300 --timeout-method thread -m gpu tests"
