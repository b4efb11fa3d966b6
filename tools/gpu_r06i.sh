#!/bin/bash
# Round 6, box 9: smoke, the default bench line, and a kernel trace of config
# 5's operator in mode 1 (the complex Arnoldi step's pass / finalize shares).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06i_c5m1
bash tools/gpu_step.sh r06i \
  "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|400|python bench.py" \
  "c5m1|300|python tools/c5_mode1.py --cycles 6 --reps 2" \
  "c5m1_trace|300|cd /tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06i_c5m1/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_mode1.py --cycles 6 --reps 1 && python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py --stats $GRAFT_REPO_ROOT/gpurun_out/r06i_c5m1/trace > $GRAFT_REPO_ROOT/gpurun_out/r06i_c5m1/kernel_stats.csv && rm -rf $GRAFT_REPO_ROOT/gpurun_out/r06i_c5m1/trace"
