set -o pipefail
mkdir -p gpurun_out
AB_ARGS="--rows 1250000 --steps 30 --warmup 3" bash tools/ab_bench.sh "a_s8nt AHIP_V_POLICY=nt" "a_s8pl AHIP_V_POLICY=plain" "b_s8nt AHIP_V_POLICY=nt" "b_s8pl AHIP_V_POLICY=plain" "c_s8nt AHIP_V_POLICY=nt" "c_s8pl AHIP_V_POLICY=plain" &&
AB_ARGS="--rows 1600000 --steps 30 --warmup 3" bash tools/ab_bench.sh "a_s16nt AHIP_V_POLICY=nt" "a_s16pl AHIP_V_POLICY=plain" "b_s16nt AHIP_V_POLICY=nt" "b_s16pl AHIP_V_POLICY=plain"
