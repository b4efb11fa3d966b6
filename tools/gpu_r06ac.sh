#!/bin/bash
# Round 6, box 28: six entries a lane at 1,024-thread complex tiles as the
# default -- the complex suites, the tile-size parity test and the
# deterministic suite on it, then U = 4 vs 6 again on one box.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06ac \
  "ztests|700|$T tests/test_gpu_z.py tests/test_gpu_zshift.py tests/test_gpu_zfold.py tests/test_gpu_zfuse.py tests/test_gpu_zgen.py tests/test_gpu_ztraj.py tests/test_gpu_ztile_threads.py tests/test_gpu_deterministic.py tests/test_gpu_fullsize.py -k 'z or c5 or determin or fixed or tile'" \
  "ab|400|VAR=AHIP_ZTILE_U VALS='4 6 4 6' bash tools/ab_c5_pack.sh r06ac_u"
