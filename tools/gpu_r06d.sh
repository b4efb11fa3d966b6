#!/bin/bash
# Round 6, box 4: the packed tiles with the DPP scan (A/B against the 20-B
# form), then the whole GPU suite on the round-6 tree.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06d \
  "ztests|300|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_z.py" \
  "ab_pack|600|bash tools/ab_c5_pack.sh r06d_pk" \
  "suite|1000|python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests"
