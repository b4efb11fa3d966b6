#!/bin/bash
# Round 6, box 35: an eighth of the row cap for the finalize-carrying first
# superblock (AHIP_LIGHT_SB=8) vs the default half, configs 2 and 3.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_step.sh r06ak \
  "ab|700|for lb in 1 8 1 8; do AHIP_LIGHT_SB=\$lb timeout -k 10 150 python3 tools/bench_configs.py C2 C3 > gpurun_out/r06ak_cfg_\$lb.json || exit 1; python3 -c \"import json;[print('LIGHT_SB=\$lb', k, round(v['best']['iters_per_s'],1), round(v['best']['spmv_plus_orth_frac'],3), {n:round(x['ms']/max(x['launches'],1)*1e3,1) for n,x in v['full_storage']['roofline']['kernels'].items()}) for l in open('gpurun_out/r06ak_cfg_\$lb.json') for k,v in json.loads(l).items()]\" || exit 1; done"
