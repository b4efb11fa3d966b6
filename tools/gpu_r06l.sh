#!/bin/bash
# Round 6, box 12: the fold passes with each row over 2-4 lanes -- tests, then
# config 5's mode-1 solve against the previous build (one-lane rows), alternating.
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
PREV=$GRAFT_REPO_ROOT/arpack-ng_amd/libarpack_hip_prev.so
bash tools/gpu_step.sh r06l \
  "ztests|500|$T tests/test_gpu_zfold.py tests/test_gpu_z.py tests/test_gpu_ztraj.py tests/test_gpu_zfuse.py tests/test_gpu_fullsize.py -k 'zfold or zrandom or zcsr or ztraj or ncv40 or c5_znaupd_zrandom'" \
  "ab1|120|python tools/c5_mode1.py --cycles 6 --reps 2" \
  "ab2|120|ARPACK_HIP_LIB=$PREV python tools/c5_mode1.py --cycles 6 --reps 2" \
  "ab3|120|python tools/c5_mode1.py --cycles 6 --reps 2" \
  "ab4|120|ARPACK_HIP_LIB=$PREV python tools/c5_mode1.py --cycles 6 --reps 2"
