#!/bin/bash
# Round-5 final tree: full GPU suite, smoke, bench, config sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_full.sh r05o || exit 1
timeout -k 10 400 python3 tools/bench_configs.py > gpurun_out/r05o_configs.json 2> gpurun_out/r05o_configs.err || { tail -20 gpurun_out/r05o_configs.err; exit 1; }
echo configs done
