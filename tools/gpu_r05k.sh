#!/bin/bash
# Round-5 measurements: V-load policy at the rank share, the rank-share sweep
# (scaling estimate) and the overlapped distributed SpMV on a 1-rank RCCL
# communicator at the share.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_env_share.sh AHIP_V_POLICY "plain nt plain nt" r05k_vpol > gpurun_out/r05k_vpol.log 2>&1 || exit 1
bash tools/gpu_shares.sh r05k > gpurun_out/r05k_shares.log 2>&1 || exit 1
for v in 0 1 0 1; do
  AHIP_DIST_OVERLAP=$v timeout -k 10 200 python3 bench.py --rows 1250000 --steps 20 --warmup 5 --no-cpu-baseline --no-ttc --no-full-storage --steady-cycles 0 --force-dist > gpurun_out/r05k_ov_$v.json 2> gpurun_out/r05k_ov.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r05k_ov_$v.json'));print('AHIP_DIST_OVERLAP=$v', round(d['value'],1))" >> gpurun_out/r05k_overlap.log
done
