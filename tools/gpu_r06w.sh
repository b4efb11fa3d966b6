#!/bin/bash
# Round 6, box 22: 1,024-thread complex tiles as the default -- the complex
# suites and config 5's full-size pins on it, then a mode-1 A/B (the plain
# product) against 256 threads on the same box.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06w \
  "ztests|600|$T tests/test_gpu_z.py tests/test_gpu_zshift.py tests/test_gpu_zfold.py tests/test_gpu_zfuse.py tests/test_gpu_zgen.py tests/test_gpu_ztraj.py tests/test_gpu_fullsize.py -k 'z or c5'" \
  "m1ab|400|for t in 256 1024 256 1024; do echo AHIP_ZTILE_T=\$t; AHIP_ZTILE_T=\$t timeout -k 10 90 python3 tools/c5_mode1.py --cycles 6 --reps 2 || exit 1; done"
