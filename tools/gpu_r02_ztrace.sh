set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_c5 -o run --output-format csv -- python3 tools/bench_configs.py C5 > gpurun_out/tr_c5.json 2>&1
