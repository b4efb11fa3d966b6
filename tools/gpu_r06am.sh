#!/bin/bash
# Round 6, box 37: the final tree's default bench line and the config-4 line.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06am \
  "bench|400|python bench.py > gpurun_out/r06am_bench.json" \
  "lap3d|400|python bench.py --workload lap3d > gpurun_out/r06am_bench_lap3d.json"
