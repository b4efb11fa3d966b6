set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err &&
timeout -k 10 200 python bench.py --rows 1250000 --steps 20 --warmup 3 --no-cpu-baseline --no-ttc --no-full-storage > gpurun_out/r02_share8.json 2>&1 &&
timeout -k 10 200 python bench.py --rows 1250000 --steps 20 --warmup 3 --no-cpu-baseline --no-ttc --no-full-storage --force-dist > gpurun_out/r02_share8_dist.json 2>&1
