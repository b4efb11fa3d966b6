#!/bin/bash
# Round profile set for a bench workload (MI355X_MICROARCH.md HBM/rocprofv3 recipe):
# one kernel-trace pass (per-kernel durations) and two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE do not fit one TCC pass), then the summaries.
#   tools/profile_round.sh TAG [bench args...]  -> gpurun_out/TAG/{pmc.json,kernel_stats.csv}
# The bench line of the trace pass names the workload (operator, n, nnz,
# storage, mode); it is written into pmc.json's "workload" block, so bench.py
# uses the summary's traffic only for a line of that same workload.  Only the
# line's own SpMV form runs (--no-full-storage: no companion measurements).
set -o pipefail
TAG=${1:-r01}
shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS="$ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ttc --no-full-storage $*"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 $ARGS \
    > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run -- python3 $ARGS \
    > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run -- python3 $ARGS \
    > "$OUT/write.log" 2>&1 || exit $?
WL=$(python3 - "$OUT/trace.log" "$ARGS" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
c = d["config"]
print(json.dumps(dict(workload=c.get("workload_key", "ns"), n=c["n"], nnz=c["nnz"],
                      storage=d["storage"], spmv_form=c.get("spmv_form"),
                      deterministic=bool(c.get("deterministic_mode")),
                      command="python3 " + sys.argv[2].replace(sys.argv[2].split()[0], "bench.py", 1))))
EOF
) || exit 1
python3 "$ROOT/tools/pmc_summary.py" --workload "$WL" "$OUT/fetch" "$OUT/write" "$OUT/trace" > "$OUT/pmc.json" &&
python3 "$ROOT/tools/pmc_summary.py" --stats "$OUT/trace" > "$OUT/kernel_stats.csv" &&
# the raw rocprofv3 output stays on the box (gpurun_out/ travels back only below 64 MiB)
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write"
