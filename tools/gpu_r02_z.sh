set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -k "z or single or large_ncv or edge or fullsize or modes" tests > gpurun_out/z_tests.log 2>&1
tail -15 gpurun_out/z_tests.log
timeout -k 10 200 python3 tools/bench_configs.py C5 > gpurun_out/z_c5.json 2>&1 &&
AHIP_ZHOST=1 timeout -k 10 200 python3 tools/bench_configs.py C5 > gpurun_out/z_c5_host.json 2>&1
tail -1 gpurun_out/z_c5.json; tail -1 gpurun_out/z_c5_host.json
