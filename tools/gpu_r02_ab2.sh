set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/bench_configs.py C2 C3 > gpurun_out/ab2_cfg.json 2>&1 &&
AB_ARGS="--rows 1250000 --steps 20 --warmup 3" bash tools/ab_bench.sh "s8auto" "s8nt AHIP_V_POLICY=nt" &&
AB_ARGS="--rows 2500000 --steps 20 --warmup 3" bash tools/ab_bench.sh "s4auto" "s4plain AHIP_V_POLICY=plain" &&
bash tools/ab_bench.sh "n1auto" &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dgks.py tests/test_gpu_ns.py > gpurun_out/ab2_tests.log 2>&1
