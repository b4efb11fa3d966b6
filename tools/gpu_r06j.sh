#!/bin/bash
# Round 6, box 10: the folded complex Arnoldi step -- its tests, the complex
# suites around it, config 5's mode-1 solve folded vs unfolded (alternating).
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06j \
  "zfold|400|$T tests/test_gpu_zfold.py" \
  "ztests|600|$T tests/test_gpu_z.py tests/test_gpu_ztraj.py tests/test_gpu_zfuse.py tests/test_gpu_zshift.py tests/test_gpu_zgen.py tests/test_gpu_fullsize.py -k 'z or c5'" \
  "ab|400|for v in 1 0 1 0; do AHIP_ZFOLD=\$v python tools/c5_mode1.py --cycles 6 --reps 2 | sed \"s/^/ZFOLD=\$v /\"; done"
