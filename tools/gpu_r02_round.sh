set -o pipefail
TAG=${1:-r02a}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_edge.py > gpurun_out/${TAG}_edge.log 2>&1 || { tail -30 gpurun_out/${TAG}_edge.log; exit 1; }
tail -2 gpurun_out/${TAG}_edge.log
bash tools/profile_round.sh $TAG || exit 1
cp gpurun_out/$TAG/pmc.json profiles/${TAG}_pmc.json
cp gpurun_out/$TAG/kernel_stats.csv profiles/${TAG}_kernel_stats.csv
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
