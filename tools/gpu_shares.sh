# Rank-share cycle rates of the folded build (scaling estimate) and the cost of
# the distributed machinery on a 1-rank RCCL communicator.
set -o pipefail
TAG=${1:-shares}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rows in 10000000 5000000 2500000 1250000; do
  for fd in "" "--force-dist"; do
    timeout -k 10 200 python3 bench.py --rows $rows --steps 20 --warmup 5 --no-cpu-baseline --no-full-storage --no-ttc $fd > gpurun_out/${TAG}_share_${rows}${fd}.json 2> gpurun_out/${TAG}_share.err || { tail -20 gpurun_out/${TAG}_share.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_share_${rows}${fd}.json'));print($rows, '$fd', round(d['value'],1), round(d['lanczos_steps_per_s']))"
  done
done
