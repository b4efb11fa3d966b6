#!/bin/bash
# The whole GPU suite with deterministic mode on at load (ARPACK_HIP_DETERMINISTIC=1):
# every solve through the fixed-point symmetric kernel / complex tiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ARPACK_HIP_DETERMINISTIC=1 timeout -k 10 900 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/${1:-detsuite}_gputests.log 2>&1
rc=$?
tail -15 gpurun_out/${1:-detsuite}_gputests.log
exit $rc
