#!/bin/bash
# Round 6, box 5: the packed tiles' entries in flight (4 vs 8), the profile
# sets of the round-6 defaults (north star with the fixed-point accumulator,
# config 5 with packed tiles), the other configs, and the 8-way share against
# the north star, alternating.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06e \
  "ab_u|600|VAR=AHIP_ZTILE_U VALS='4 8 4 8' bash tools/ab_c5_pack.sh r06e_u" \
  "prof_ns|900|bash tools/profile_round.sh r06e_ns" \
  "prof_c5|600|bash tools/profile_c5.sh r06e_c5" \
  "configs|900|python3 tools/bench_configs.py > gpurun_out/r06e_configs.json" \
  "shares|600|for r in 1250000 10000000 1250000 10000000; do python3 bench.py --rows \$r --steps 20 --warmup 5 --no-cpu-baseline --no-ttc --no-full-storage --steady-cycles 0 > gpurun_out/r06e_share_\$r.json && python3 -c \"import json;d=json.load(open('gpurun_out/r06e_share_\$r.json'));print(\$r, round(d['value'],2), d['config']['spmv_form'])\" || exit 1; done"
