#!/bin/bash
# Run GPU steps in order, each under its own time limit; a test failure
# (exit 1) does not stop the sequence, anything that looks like a fault, an
# abort, a crash or a time limit (any other non-zero status) ends it there.
#   bash tools/gpu_step.sh TAG "name|seconds|command" ...
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/${TAG}_${name}.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -3 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping after $name (rc $rc)"
    exit $rc
  fi
done
