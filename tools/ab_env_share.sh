#!/bin/bash
# Same-box A/B of an environment knob on the bench at one rank's share of the
# north star (1.25e6 rows, single GPU):  bash tools/ab_env_share.sh VAR "v1 v2 v1 v2" TAG [rows]
set -o pipefail
VAR=$1; VALS=$2; TAG=${3:-abs}; ROWS=${4:-1250000}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
i=0
for v in $VALS; do
  i=$((i + 1))
  out=gpurun_out/${TAG}_${i}_$v.json
  env $VAR=$v timeout -k 10 200 python3 bench.py --rows $ROWS --steps 20 --warmup 5 --no-cpu-baseline --no-ttc --no-full-storage --steady-cycles 0 > $out 2>gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out'));print('$VAR=$v', round(d['value'],2), {k:(v['launches'], round(v['ms']/max(v['launches'],1)*1e3,1)) for k,v in d['kernels'].items() if v['launches']})"
done
