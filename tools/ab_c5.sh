# Complex-engine change check: complex parity tests, then a same-box A/B of the
# C5 operator in mode 1 and mode 3 against a previous build
# (arpack-ng_amd/libarpack_hip_prev.so):  bash tools/ab_c5.sh TAG
set -o pipefail
TAG=${1:-abc5}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_zfuse.py tests/test_gpu_z.py tests/test_gpu_zshift.py tests/test_gpu_single.py tests/test_gpu_large_ncv.py \
  "tests/test_gpu_fullsize.py::test_c5_znaupd_zrandom_full_size" \
  "tests/test_gpu_fullsize.py::test_c5_znaupd_shift_invert_full_size" \
  > gpurun_out/${TAG}_ztests.log 2>&1 || { tail -40 gpurun_out/${TAG}_ztests.log; exit 1; }
tail -2 gpurun_out/${TAG}_ztests.log
PREV=$GRAFT_REPO_ROOT/arpack-ng_amd/libarpack_hip_prev.so
for lib in prev new prev new; do
  if [ $lib = prev ]; then L=$PREV; else L=; fi
  ARPACK_HIP_LIB=$L timeout -k 10 120 python3 tools/c5_mode1.py >> gpurun_out/${TAG}_mode1.jsonl 2>>gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  echo "$lib $(tail -1 gpurun_out/${TAG}_mode1.jsonl)"
done
for lib in prev new; do
  if [ $lib = prev ]; then L=$PREV; else L=; fi
  ARPACK_HIP_LIB=$L timeout -k 10 120 python3 tools/c5_mode3.py --cycles 5 >> gpurun_out/${TAG}_mode3.jsonl 2>>gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  echo "$lib $(tail -1 gpurun_out/${TAG}_mode3.jsonl | cut -c1-400)"
done
