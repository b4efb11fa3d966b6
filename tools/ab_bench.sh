#!/bin/bash
# A/B of engine tuning knobs / library builds in ONE process per variant on the same box:
#   bash tools/ab_bench.sh "tag1 VAR=.. VAR=.." "tag2 VAR=.." ...
# (ARPACK_HIP_LIB=path selects another build of the library); AB_ARGS adds bench
# arguments (e.g. --rows 1250000).  Prints "tag iters/s ms/cycle" per variant.
mkdir -p gpurun_out
for spec in "$@"; do
  set -- $spec
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-ttc --no-full-storage --no-profile ${AB_ARGS:-} \
      > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print('$tag', round(d['value'],3), round(d['ms_per_step'],3))"
done
