# Folded DGKS steps: GPU suite, then bench with and without folding (same box).
set -o pipefail
TAG=${1:-r02d}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputests.log
for f in 1 0 1; do
  AHIP_FOLD=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-storage > gpurun_out/${TAG}_bench_fold$f.json 2> gpurun_out/${TAG}_bench_fold$f.err || { tail -20 gpurun_out/${TAG}_bench_fold$f.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/${TAG}_bench_fold$f.json'));print('fold=$f', round(d['value'],2), d['time_to_converge'], {k:(round(v['ms'],1),v['launches']) for k,v in d['kernels'].items()})"
done
