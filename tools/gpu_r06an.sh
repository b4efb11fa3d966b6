#!/bin/bash
# Round 6, box 38: configs 2 and 3's profile set on the final tree (kernel trace
# + FETCH_SIZE / WRITE_SIZE passes); the raw traces stay on the box.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06an \
  "prof_c23|900|bash tools/profile_c23.sh r06an_c23 && rm -rf gpurun_out/r06an_c23/trace gpurun_out/r06an_c23/fetch gpurun_out/r06an_c23/write"
