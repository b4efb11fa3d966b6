# Column alignment of V: the bench at n = 10^7 (columns 128-B aligned) and at
# n = 10^7 - 1 (odd: column starts off 128 B), alternating:  bash tools/ab_align.sh TAG
set -o pipefail
TAG=${1:-align}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 10000000 9999999 10000000 9999999; do
  timeout -k 10 200 python3 bench.py --n $n --steps 10 --warmup 3 --no-cpu-baseline --no-full-storage --no-ttc > gpurun_out/${TAG}_$n.json 2>gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_$n.json'));print('n=$n', round(d['value'],2), {k:(round(v['ms']/max(v['launches'],1)*1e3,1), round(v['gbs'] or 0)) for k,v in d['kernels'].items()})" | tee -a gpurun_out/${TAG}_summary.txt
done
