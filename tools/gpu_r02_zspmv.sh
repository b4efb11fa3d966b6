set -o pipefail
mkdir -p gpurun_out
for g in 0 8 16 32 64 auto; do
  if [ $g = auto ]; then timeout -k 10 120 python3 tools/zspmv_time.py >> gpurun_out/zspmv.jsonl 2>&1 || exit 1;
  else AHIP_ZCSR_G=$g timeout -k 10 120 python3 tools/zspmv_time.py >> gpurun_out/zspmv.jsonl 2>&1 || exit 1; fi
done
