#!/bin/bash
# Round 6, box 6: the profile sets of the round-6 defaults (raw traces removed
# on the box), the dynamic-range guard's tests, and the share's accumulator A/B.
cd "$GRAFT_REPO_ROOT"
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
bash tools/gpu_step.sh r06f \
  "symtests|400|$T tests/test_gpu_symspmv.py tests/test_gpu_bench_contract.py -k 'graded or lap3d or matches_full'" \
  "prof_ns|900|bash tools/profile_round.sh r06f_ns" \
  "prof_c5|600|bash tools/profile_c5.sh r06f_c5" \
  "acc_share|400|for a in fixed fp64 fixed fp64; do python3 bench.py --rows 1250000 --sym-acc \$a --steps 20 --warmup 5 --no-cpu-baseline --no-ttc --no-full-storage --steady-cycles 0 > gpurun_out/r06f_acc_\$a.json && python3 -c \"import json;d=json.load(open('gpurun_out/r06f_acc_\$a.json'));print('\$a', round(d['value'],2), d['config']['spmv_form'], {k:(v['launches'], round(v['ms']/max(v['launches'],1)*1e3,1)) for k,v in d['kernels'].items() if v['launches']})\" || exit 1; done"
