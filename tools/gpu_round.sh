# Round profile set of the folded build: new fold tests, bench at the driver's
# settings, kernel trace + PMC passes (tools/profile_round.sh), config sweep.
set -o pipefail
TAG=${1:-round}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fold.py > gpurun_out/${TAG}_fold_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_fold_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_fold_tests.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
bash tools/profile_round.sh $TAG || exit 1
timeout -k 10 300 python3 tools/bench_configs.py > gpurun_out/${TAG}_configs.json 2> gpurun_out/${TAG}_configs.err || { tail -20 gpurun_out/${TAG}_configs.err; exit 1; }
cat gpurun_out/${TAG}_configs.json
