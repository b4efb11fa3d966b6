#!/bin/bash
# Round 6, box 13: where config 5's mode-1 cycle waits on the host -- kernel
# trace of two solves, gap summary from the first start vector on.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06m_c5m1
mkdir -p $O
bash tools/gpu_step.sh r06m \
  "trace|300|cd /tmp && rocprofv3 --kernel-trace -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_mode1.py --cycles 6 --reps 1 && python3 $GRAFT_REPO_ROOT/tools/gap_summary.py $O/trace --from k_larnv > $O/gaps.txt && rm -rf $O/trace"
