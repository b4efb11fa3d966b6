#!/bin/bash
# Round 6, box 2: the unified symmetric walk (one kernel, two accumulators),
# its hand-off orderings, the light-superblock variants; parity then A/B.
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06b \
  "sym|600|$T tests/test_gpu_symspmv.py tests/test_gpu_symspmv_handoff.py tests/test_gpu_deterministic.py tests/test_gpu_bench_contract.py" \
  "gen|300|$T tests/test_gpu_gen.py tests/test_gpu_modes.py" \
  "ztests|600|$T tests/test_gpu_z.py tests/test_gpu_zshift.py tests/test_gpu_zfuse.py tests/test_gpu_deterministic.py -k 'zcsr or zshift or zfuse or complex or ztile or Z'" \
  "ab_pack|600|bash tools/ab_c5_pack.sh r06b_pk" \
  "handoff2|300|AHIP_HANDOFF=2 $T tests/test_gpu_symspmv_handoff.py tests/test_gpu_deterministic.py -k 'handoff or uneven or wide'" \
  "ns_full|600|$T tests/test_gpu_fullsize.py -k north_star" \
  "ab_handoff_ns|600|bash tools/ab_env_share.sh AHIP_HANDOFF '1 2 1 2 1 2' r06b_hns 10000000" \
  "ab_handoff_share|400|bash tools/ab_env_share.sh AHIP_HANDOFF '1 2 1 2 1 2' r06b_hsh 1250000" \
  "ab_light_ns|600|bash tools/ab_env_share.sh AHIP_LIGHT_SB '1 2 1 2' r06b_lns 10000000" \
  "ab_light_share|400|bash tools/ab_env_share.sh AHIP_LIGHT_SB '1 2 1 2 0' r06b_lsh 1250000"
