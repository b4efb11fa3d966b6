#!/bin/bash
# Round 6, box 11: two column slices for the complex tiles (AHIP_ZSLICES=2:
# half the partial-sum traffic of 4) -- correctness on the split tests, then a
# same-box A/B on config 5 in mode 3; the folded mode-1 kernel trace.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
mkdir -p gpurun_out/r06k_c5m1
bash tools/gpu_step.sh r06k \
  "zs2|300|AHIP_ZSLICES=2 $T tests/test_gpu_z.py tests/test_gpu_zshift.py -k 'split or shift or zcsr'" \
  "ab|700|VAR=AHIP_ZSLICES VALS='4 2 4 2' bash tools/ab_c5_pack.sh r06k_slices" \
  "c5m1_trace|300|cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06k_c5m1/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_mode1.py --cycles 6 --reps 1 && python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py --stats $GRAFT_REPO_ROOT/gpurun_out/r06k_c5m1/trace > $GRAFT_REPO_ROOT/gpurun_out/r06k_c5m1/kernel_stats.csv && rm -rf $GRAFT_REPO_ROOT/gpurun_out/r06k_c5m1/trace"
