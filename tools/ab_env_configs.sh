#!/bin/bash
# Same-box A/B of an environment knob on BASELINE configs 2-4 (tools/bench_configs.py):
#   bash tools/ab_env_configs.sh VAR "v1 v2 v1 v2" TAG [configs...]
# prints per run: cycles/s per storage and the average finalize launch (us).
set -o pipefail
VAR=$1; VALS=$2; TAG=$3; shift 3
CFG=${*:-C2 C3}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
i=0
for v in $VALS; do
  i=$((i + 1))
  out=gpurun_out/${TAG}_${i}_$v.json
  env $VAR=$v timeout -k 10 300 python3 tools/bench_configs.py $CFG > $out 2> gpurun_out/${TAG}.err \
    || { echo "$VAR=$v failed"; tail -20 gpurun_out/${TAG}.err; exit 1; }
  python3 - "$out" "$VAR=$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for name, rec in d.items():
    for st in ("full_storage", "sym_storage"):
        r = rec.get(st)
        if not isinstance(r, dict):
            continue
        k = r.get("roofline", {}).get("kernels", {})
        f = k.get("finalize", {})
        sp = k.get("spmv", {})
        print(sys.argv[2], name[:2], st[:4], "%.1f cycles/s" % r["iters_per_s"],
              "finalize %d x %.2f us" % (f["launches"], 1e3 * f["ms"] / f["launches"]) if f.get("launches") else "",
              "spmv %.1f us" % (1e3 * sp["ms"] / sp["launches"]) if sp.get("launches") else "")
PY
done
