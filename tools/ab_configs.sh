#!/bin/bash
# Same-box A/B of library builds on BASELINE configs 2 and 3 (n = 1e6), where the
# per-step fixed costs (finalize launches) show:
#   bash tools/ab_configs.sh TAG libA.so libB.so [configs...]
# Alternates A, B, A, B; prints per run: cycles/s (full and symmetric storage)
# and the average finalize launch (us) from the kernel-mode hipEvent profile.
set -o pipefail
TAG=$1; LA=$2; LB=$3; shift 3
CFG=${*:-C2 C3}
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for v in A B; do
    lib=$LA; [ $v = B ] && lib=$LB
    out=gpurun_out/${TAG}_${v}${rep}.json
    ARPACK_HIP_LIB=$lib timeout -k 10 300 python3 tools/bench_configs.py $CFG > $out 2> gpurun_out/${TAG}.err \
      || { echo "$v$rep failed"; tail -20 gpurun_out/${TAG}.err; exit 1; }
    python3 - "$out" "$v$rep" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
for name, rec in d.items():
    for st in ("full_storage", "sym_storage"):
        r = rec.get(st)
        if not isinstance(r, dict):
            continue
        k = r.get("roofline", {}).get("kernels", {})
        f = k.get("finalize", {})
        fin = 1e3 * f["ms"] / f["launches"] if f.get("launches") else None
        print(sys.argv[2], name[:2], st[:4], "%.1f cycles/s" % r["iters_per_s"],
              "finalize %.2f us" % fin if fin else "",
              "spmv+orth frac %.3f" % r["roofline"]["spmv_plus_orth_frac"] if "roofline" in r else "")
EOF
  done
done
