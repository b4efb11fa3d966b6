#!/bin/bash
# Round 6, first box: the new bench routes (lap3d, comm profile, workload-keyed
# PMC), the deterministic fallback, the P = 8 config-4 rehearsal; then the
# NS and lap3d bench lines and their profile sets.
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06a \
  "contract|600|$T tests/test_gpu_bench_contract.py tests/test_gpu_deterministic.py" \
  "dist|900|$T tests/test_gpu_dist.py -k 'lap3d or symmetric_storage or mode_agreed'" \
  "bench_ns|400|python3 bench.py --steps 20 --warmup 5 > gpurun_out/r06a_bench_ns.json" \
  "bench_lap3d|400|python3 bench.py --workload lap3d --steps 20 --warmup 5 > gpurun_out/r06a_bench_lap3d.json" \
  "prof_ns|900|bash tools/profile_round.sh r06a_ns" \
  "prof_lap3d|900|bash tools/profile_round.sh r06a_lap3d --workload lap3d" \
  "force_dist|400|python3 bench.py --steps 10 --warmup 2 --force-dist --no-cpu-baseline --no-full-storage > gpurun_out/r06a_force_dist.json"
