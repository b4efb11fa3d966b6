set -o pipefail
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/arpack-ng_amd/ab_plainv.so
for rep in 1 2; do
timeout -k 10 200 python3 tools/bench_configs.py C2 C3 > gpurun_out/ab1_cfg_nt_$rep.json 2>&1 &&
ARPACK_HIP_LIB=$L timeout -k 10 200 python3 tools/bench_configs.py C2 C3 > gpurun_out/ab1_cfg_pv_$rep.json 2>&1 || exit 1
done
AB_ARGS="--rows 1250000 --steps 20 --warmup 3" bash tools/ab_bench.sh "s8nt" "s8pv ARPACK_HIP_LIB=$L" "s8nt2" "s8pv2 ARPACK_HIP_LIB=$L" &&
AB_ARGS="--rows 2500000 --steps 20 --warmup 3" bash tools/ab_bench.sh "s4nt" "s4pv ARPACK_HIP_LIB=$L" &&
bash tools/ab_bench.sh "n1nt" "n1pv ARPACK_HIP_LIB=$L"
