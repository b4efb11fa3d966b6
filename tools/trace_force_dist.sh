#!/bin/bash
# Kernel traces of the rank-share bench, single-GPU engine vs the 1-rank
# distributed path (--force-dist):  tools/trace_force_dist.sh TAG
set -o pipefail
TAG=${1:-fd}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="$ROOT/bench.py --rows 1250000 --steps 40 --warmup 5 --no-cpu-baseline --no-ttc --no-full-storage --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/plain" -o run -- python3 $ARGS > "$OUT/plain.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/fd" -o run -- python3 $ARGS --force-dist > "$OUT/fd.log" 2>&1 || exit $?
python3 "$ROOT/tools/pmc_summary.py" --stats "$OUT/plain" > "$OUT/plain_stats.csv" &&
python3 "$ROOT/tools/pmc_summary.py" --stats "$OUT/fd" > "$OUT/fd_stats.csv"
