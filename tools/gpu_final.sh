# Final-tree numbers: bench at the driver's settings and the config sweep.
set -o pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.json
timeout -k 10 400 python3 tools/bench_configs.py > gpurun_out/${TAG}_configs.json 2> gpurun_out/${TAG}_configs.err || { tail -20 gpurun_out/${TAG}_configs.err; exit 1; }
echo configs done
