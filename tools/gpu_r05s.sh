#!/bin/bash
# Round-5 final profile set (kernel trace + PMC passes) and the bench line with
# its deterministic-mode companion.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05s_bench.json 2> gpurun_out/r05s_bench.err || { tail -20 gpurun_out/r05s_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r05s_bench.json'));print(d['value'], d['full_storage'], d['deterministic'], d['roofline']['frac'])"
bash tools/profile_round.sh r05s || exit 1
head -12 gpurun_out/r05s/kernel_stats.csv | cut -c1-160
