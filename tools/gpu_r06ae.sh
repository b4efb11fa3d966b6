#!/bin/bash
# Round 6, box 30: the final tree's measurements -- BASELINE configs 2-5
# (tools/bench_configs.py), the default bench line, the config-4 bench line.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06ae \
  "configs|600|python tools/bench_configs.py > gpurun_out/r06ae_configs.json" \
  "bench|400|python bench.py > gpurun_out/r06ae_bench.json" \
  "lap3d|400|python bench.py --workload lap3d > gpurun_out/r06ae_bench_lap3d.json"
