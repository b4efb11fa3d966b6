# Same-box A/B of an environment knob on the bench: bash tools/ab_env.sh VAR "v1 v2 v1 v2" TAG
# (EXTRA="--rows 1250000" adds bench arguments; STEPS sets the timed steps)
set -o pipefail
VAR=$1; VALS=$2; TAG=${3:-ab}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for v in $VALS; do
  i=$((i + 1))
  out=gpurun_out/${TAG}_${i}_$v.json
  env $VAR=$v timeout -k 10 200 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-full-storage --no-ttc $EXTRA > $out 2>gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out'));print('$VAR=$v', round(d['value'],2), {k:(round(v['ms']/max(v['launches'],1)*1e3,1)) for k,v in d['kernels'].items()})"
done
