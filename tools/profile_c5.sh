#!/bin/bash
# Profile set for BASELINE config 5 in shift-invert mode 3 (tools/c5_mode3.py:
# znaupd + the device BiCGStab): one kernel-trace pass and separate FETCH_SIZE /
# WRITE_SIZE PMC passes (MI355X_MICROARCH.md recipe), then the summaries.
#   tools/profile_c5.sh TAG      -> gpurun_out/TAG/{pmc.json,kernel_stats.csv}
set -o pipefail
TAG=${1:-r03_c5}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="$ROOT/tools/c5_mode3.py --cycles 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 $ARGS \
    > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 $ARGS \
    > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 $ARGS \
    > "$OUT/write.log" 2>&1 || exit $?
python3 "$ROOT/tools/pmc_summary.py" --workload "{\"workload\": \"c5_mode3\", \"n\": 500000, \"command\": \"python3 tools/c5_mode3.py --cycles 2\"}" "$OUT/fetch" "$OUT/write" "$OUT/trace" > "$OUT/pmc.json" &&
python3 "$ROOT/tools/pmc_summary.py" --stats "$OUT/trace" > "$OUT/kernel_stats.csv" &&
# the raw rocprofv3 output stays on the box (gpurun_out/ travels back only below 64 MiB)
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write"
