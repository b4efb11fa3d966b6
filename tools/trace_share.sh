#!/bin/bash
# Kernel trace + gap summary of the bench at one rank's share of the north star
# (1.25e6 rows) and at full size:  tools/trace_share.sh TAG
set -o pipefail
TAG=${1:-share}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for rows in 1250000 10000000; do
  ARGS="$ROOT/bench.py --rows $rows --steps 10 --warmup 3 --no-cpu-baseline --no-ttc --no-full-storage --no-profile --steady-cycles 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/r$rows" -o run -- python3 $ARGS > "$OUT/r$rows.log" 2>&1 || exit $?
  python3 "$ROOT/tools/pmc_summary.py" --stats "$OUT/r$rows" > "$OUT/r${rows}_stats.csv" || exit 1
  python3 "$ROOT/tools/gap_summary.py" "$OUT/r$rows" --from k_vq_update > "$OUT/r${rows}_gaps.txt" 2>&1 || exit 1
done
