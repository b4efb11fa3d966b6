#!/bin/bash
# Round 6, box 36: an eighth of the row cap for the finalize-carrying first
# superblock as the default -- configs 2-4 on it, then the full GPU suite and
# smoke.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06al \
  "configs|400|timeout -k 10 300 python tools/bench_configs.py C2 C3 C4 > gpurun_out/r06al_configs.json" \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "suite|1000|python -u -m pytest -v --durations=20 --timeout 300 --timeout-method thread -m gpu tests"
