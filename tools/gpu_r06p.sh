#!/bin/bash
# Round 6, box 16: the folded complex step on a 3-eigenvalue operator (Krylov
# spaces that close: parks, give-ups, restarts inside folded cycles); a lighter
# first superblock for the full-storage SELL kernel's finalize-carrying
# workgroup (AHIP_LIGHT_SB=4: a quarter of the row cap instead of half), C2/C3.
cd "$GRAFT_REPO_ROOT"
C="python tools/bench_configs.py"
bash tools/gpu_step.sh r06p \
  "zfold|300|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_zfold.py" \
  "c3a|200|$C C3 > gpurun_out/r06p_c3_lsb2a.json" \
  "c3b|200|AHIP_LIGHT_SB=4 $C C3 > gpurun_out/r06p_c3_lsb4a.json" \
  "c3c|200|$C C3 > gpurun_out/r06p_c3_lsb2b.json" \
  "c3d|200|AHIP_LIGHT_SB=4 $C C3 > gpurun_out/r06p_c3_lsb4b.json" \
  "c2a|200|$C C2 > gpurun_out/r06p_c2_lsb2a.json" \
  "c2b|200|AHIP_LIGHT_SB=4 $C C2 > gpurun_out/r06p_c2_lsb4a.json"
