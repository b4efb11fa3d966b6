#!/bin/bash
# Round 6, box 24: BiCGStab vector kernels at 1,024 threads a block (16 waves
# instead of 4 under the same 512-block partial grid; a variant build,
# -DAHIP_BI_T=1024) -- the shift-invert tests on it, then config 5 in mode 3
# against the default build on the same box.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
V=arpack-ng_amd/variants/libarpack_hip_bi1024.so
D=arpack-ng_amd/libarpack_hip.so
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06y \
  "vtests|400|ARPACK_HIP_LIB=$V $T tests/test_gpu_zshift.py tests/test_gpu_zgen.py" \
  "ab|600|VAR=ARPACK_HIP_LIB VALS='$D $V $D $V' bash tools/ab_c5_pack.sh r06y_bi"
