#!/bin/bash
# Round 6, box 29: six entries a lane for the deterministic complex tiles too --
# the tile-size parity test and the deterministic suite, then config 5 in mode
# 3 in deterministic mode, U = 4 vs 6.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06ad \
  "tests|400|$T tests/test_gpu_ztile_threads.py tests/test_gpu_deterministic.py" \
  "detab|400|ARPACK_HIP_DETERMINISTIC=1 VAR=AHIP_ZTILE_U VALS='4 6 4 6' bash tools/ab_c5_pack.sh r06ad_det"
