#!/bin/bash
# Round 6, box 34: BiCGStab vector kernels that load their first element before
# summing the previous kernel's partials -- the shift-invert tests, then config
# 5 in mode 3 against the previous build on the same box.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B=arpack-ng_amd/variants/libarpack_hip_base.so
D=arpack-ng_amd/libarpack_hip.so
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06ai \
  "tests|400|$T tests/test_gpu_zshift.py tests/test_gpu_zgen.py tests/test_gpu_gen.py" \
  "ab|600|VAR=ARPACK_HIP_LIB VALS='$B $D $B $D $B $D' bash tools/ab_c5_pack.sh r06ai_pre"
