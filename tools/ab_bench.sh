#!/bin/bash
# A/B of engine tuning knobs in ONE process per variant on the same box:
#   bash tools/ab_bench.sh "tag1 VAR=.. VAR=.." "tag2 VAR=.." ...
# prints "tag iters/s" per variant (bench.py, no CPU baseline / ttc / profiler).
mkdir -p gpurun_out
for spec in "$@"; do
  set -- $spec
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ttc --no-full-storage --no-profile ${AB_ARGS:-} \
      > gpurun_out/ab_$tag.log 2>&1 || { echo "$tag failed"; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$tag.log').read().splitlines()[-1]);print('$tag', round(d['value'],3), round(d['ms_per_step'],3))"
done
