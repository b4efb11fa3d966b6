#!/bin/bash
# Round 6, box 21: 512- and 1024-thread complex tile workgroups
# (AHIP_ZTILE_T: 4 / 8 waves a SIMD instead of 2 under the same 64 KB of LDS
# row sums) -- the split tests under each, then a same-box A/B on config 5 in
# mode 3.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06v \
  "t512|300|AHIP_ZTILE_T=512 $T tests/test_gpu_z.py tests/test_gpu_zshift.py -k 'split or shift or zcsr or tile'" \
  "t1024|300|AHIP_ZTILE_T=1024 $T tests/test_gpu_z.py tests/test_gpu_zshift.py -k 'split or shift or zcsr or tile'" \
  "ab|700|VAR=AHIP_ZTILE_T VALS='256 512 1024 256 512 1024' bash tools/ab_c5_pack.sh r06v_tt"
