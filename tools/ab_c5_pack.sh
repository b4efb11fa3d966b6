#!/bin/bash
# Same-box A/B of a complex-tile knob on config 5 in mode 3 (default: the
# packed 18-B entries vs the 20-B form, AHIP_ZTILE_PACK=0):
#   [VAR=AHIP_ZTILE_U VALS="4 8 4 8"] bash tools/ab_c5_pack.sh TAG
set -o pipefail
TAG=${1:-abpk}
V=${VAR:-AHIP_ZTILE_PACK}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VALS:-1 0 1 0}; do
  env $V=$v timeout -k 10 150 python3 tools/c5_mode3.py --cycles 5 >> gpurun_out/${TAG}_mode3.jsonl 2>>gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/${TAG}_mode3.jsonl')][-1];r=d['solver_roofline'];print('$V=$v', d['cycles'], d['opx'], 'ms/solve', round(d['ms_per_solve'],3), 'it/solve', round(d['bicgstab_iters_per_solve'],1), 'frac', round(r['frac'],3), 'B/it', r['bytes_per_iter'], 'form', r['tile_form'], 'steady', d['steady_state'] and round(d['steady_state']['cycles_per_s'],2))"
done
