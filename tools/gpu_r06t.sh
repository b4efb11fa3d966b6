#!/bin/bash
# Round 6, box 20: where the complex-shift mode-4 run departs from the reference.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_step.sh r06t "probe|200|python tools/probe_cshift.py"
