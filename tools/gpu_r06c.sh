#!/bin/bash
# Round 6, box 3: the fixed-point accumulator as the symmetric default, the
# packed complex tiles (fixed), dnaupd_gen; then the NS line, its TTC
# reproducibility, and the C5 encoding A/B.
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06c \
  "ztests|600|$T tests/test_gpu_z.py tests/test_gpu_zshift.py tests/test_gpu_zfuse.py" \
  "ab_pack|600|bash tools/ab_c5_pack.sh r06c_pk" \
  "sym|600|$T tests/test_gpu_symspmv.py tests/test_gpu_symspmv_handoff.py tests/test_gpu_deterministic.py tests/test_gpu_bench_contract.py tests/test_gpu_gen.py" \
  "dist_sym|900|$T tests/test_gpu_dist.py -k 'symmetric_storage or mode_agreed or chained'" \
  "bench_ns|400|python3 bench.py --steps 20 --warmup 5 > gpurun_out/r06c_bench.json" \
  "ttc_repeat|600|python3 tools/ttc_repeat.py --repeats 3 > gpurun_out/r06c_ttc_repeat.json"
