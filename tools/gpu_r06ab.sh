#!/bin/bash
# Round 6, box 27: entries a lane keeps in flight at 1,024-thread complex tiles
# (AHIP_ZTILE_U=6, 7, 8 (8 held to 64 VGPRs)), config 5 in mode 3, same box.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_step.sh r06ab \
  "ab|500|VAR=AHIP_ZTILE_U VALS='6 7 8 6 7 8' bash tools/ab_c5_pack.sh r06ab_u"
