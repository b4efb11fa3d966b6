set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_c2 -o run --output-format csv -- python3 tools/bench_configs.py C2 > gpurun_out/tr_c2.json 2>gpurun_out/tr_c2.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_s8 -o run --output-format csv -- python3 bench.py --rows 1250000 --steps 20 --warmup 3 --no-cpu-baseline --no-ttc --no-full-storage --no-profile > gpurun_out/tr_s8.json 2>gpurun_out/tr_s8.err &&
python3 tools/timeline.py gpurun_out/tr_c2 > gpurun_out/tl_c2.txt 2>&1 &&
python3 tools/timeline.py gpurun_out/tr_s8 > gpurun_out/tl_s8.txt 2>&1
