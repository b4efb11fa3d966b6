#!/bin/bash
# Round 6, box 31: a 512-block partial grid (AHIP_NBLK=512, default 1,024) at
# n ~ 10^6 -- configs 2 and 3 and a rank's share A/B, and the full-size pins
# of configs 2 and 3 against the reference under it (the sums' order changes).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06af \
  "pins|600|AHIP_NBLK=512 $T tests/test_gpu_fullsize.py -k 'c2 or c3'" \
  "ab|700|for nb in 1024 512 1024 512; do AHIP_NBLK=\$nb timeout -k 10 150 python3 tools/bench_configs.py C2 C3 > gpurun_out/r06af_cfg_\$nb.json || exit 1; python3 -c \"import json;[print('NBLK=\$nb', k, round(v['best']['iters_per_s'],1), round(v['best']['spmv_plus_orth_frac'],3), {n:round(x['ms']/max(x['launches'],1)*1e3,1) for n,x in v['full_storage']['roofline']['kernels'].items()}) for l in open('gpurun_out/r06af_cfg_\$nb.json') for k,v in json.loads(l).items()]\" || exit 1; AHIP_NBLK=\$nb timeout -k 10 150 python3 bench.py --rows 1250000 --steps 20 --warmup 5 --no-cpu-baseline --no-ttc --no-full-storage --steady-cycles 0 > gpurun_out/r06af_share_\$nb.json || exit 1; python3 -c \"import json;d=json.load(open('gpurun_out/r06af_share_\$nb.json'));print('NBLK=\$nb share', round(d['value'],2))\" || exit 1; done"
