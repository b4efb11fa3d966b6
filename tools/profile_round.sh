#!/bin/bash
# Round profile set for the bench workload (MI355X_MICROARCH.md HBM/rocprofv3 recipe):
# one kernel-trace pass (per-kernel durations) and two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE do not fit one TCC pass), then the summaries.
#   tools/profile_round.sh TAG        -> gpurun_out/TAG/{pmc.json,kernel_stats.csv}
set -o pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="$ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ttc"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 $ARGS \
    > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 $ARGS \
    > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 $ARGS \
    > "$OUT/write.log" 2>&1 || exit $?
python3 "$ROOT/tools/pmc_summary.py" "$OUT/fetch" "$OUT/write" "$OUT/trace" > "$OUT/pmc.json" &&
python3 "$ROOT/tools/pmc_summary.py" --stats "$OUT/trace" > "$OUT/kernel_stats.csv"
