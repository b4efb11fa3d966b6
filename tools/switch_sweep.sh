#!/bin/bash
# Engine switches (INTEGRATION.md "Engine switches") against the parity subset:
# every non-default form must still pass the fixtures the default passes.
#   tools/switch_sweep.sh TAG   -> gpurun_out/TAG_switches.log
set -o pipefail
TAG=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${TAG}_switches.log
cd "$ROOT" || exit 1
mkdir -p gpurun_out
: > "$OUT"
TESTS="tests/test_gpu_parity.py tests/test_gpu_ns.py tests/test_gpu_fold.py tests/test_gpu_z.py tests/test_gpu_modes.py tests/test_gpu_symspmv.py tests/test_gpu_zshift.py"
for sw in "AHIP_FOLD=0" "AHIP_FOLD=0 AHIP_CHAIN=0" "AHIP_FOLD_NS=0" "AHIP_FOLD_NTS=0 AHIP_VQ_NTS=0" \
          "AHIP_FUSED_FIN=0" "AHIP_ZSPLIT=0" "AHIP_ZSPLIT=csr" "AHIP_V_POLICY=plain" "AHIP_V_POLICY=nt"; do
    echo "=== $sw" >> "$OUT"
    env $sw timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS \
        >> "$OUT" 2>&1 || { echo "FAILED under $sw" >> "$OUT"; exit 1; }
done
echo "all switches green" >> "$OUT"
