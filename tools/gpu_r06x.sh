#!/bin/bash
# Round 6, box 23: the deterministic complex tiles at 1,024 threads -- the
# workgroup-size parity test, the deterministic suite, then config 5 in mode 3
# in deterministic mode at 256 vs 1,024 threads.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06x \
  "tests|400|$T tests/test_gpu_ztile_threads.py tests/test_gpu_deterministic.py" \
  "detab|500|ARPACK_HIP_DETERMINISTIC=1 VAR=AHIP_ZTILE_T VALS='256 1024 256 1024' bash tools/ab_c5_pack.sh r06x_det"
