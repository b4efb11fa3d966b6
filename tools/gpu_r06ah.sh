#!/bin/bash
# Round 6, box 33: config 5's profile set on the final tiles (1,024 threads, six
# entries a lane): kernel trace + FETCH_SIZE / WRITE_SIZE passes.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06ah \
  "prof_c5|600|bash tools/profile_c5.sh r06ah_c5"
