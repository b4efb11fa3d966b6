# Quick GPU check of a build: core parity tests, bench (no CPU baseline), and a
# rocprofv3 kernel trace of a short bench -> gpurun_out/TAG_*.
#   bash tools/gpu_quick.sh TAG [pytest files...]
set -o pipefail
TAG=${1:-quick}; shift
TESTS=${@:-tests/test_gpu_parity.py tests/test_gpu_fold.py tests/test_gpu_dgks.py tests/test_gpu_z.py}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread $TESTS > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-storage > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('bench', round(d['value'],2), 'ttc', round(d['time_to_converge']['seconds'],4), 'frac', round(d['roofline']['frac'],4), {k:(round(v['ms']/max(v['launches'],1)*1e3,1)) for k,v in d['kernels'].items()})"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ttc --no-full-storage > "$OUT.log" 2>&1 ) || exit 1
python3 tools/pmc_summary.py --stats "$OUT" > gpurun_out/${TAG}_kernel_stats.csv
