set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/chain_tests.log 2>&1
rc=$?
tail -5 gpurun_out/chain_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_ARGS="--rows 1250000 --steps 20 --warmup 3" bash tools/ab_bench.sh "s8ch" "s8noch AHIP_CHAIN=0" "s8ch2" "s8noch2 AHIP_CHAIN=0" &&
bash tools/ab_bench.sh "n1ch" "n1noch AHIP_CHAIN=0" &&
timeout -k 10 200 python3 tools/bench_configs.py C2 C3 > gpurun_out/chain_cfg.json 2>&1 &&
AHIP_CHAIN=0 timeout -k 10 200 python3 tools/bench_configs.py C2 C3 > gpurun_out/nochain_cfg.json 2>&1
