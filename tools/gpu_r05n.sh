#!/bin/bash
# Round-5 complex fixed-point tiles (k_ztile_det): the deterministic tests, the
# complex parity suites, and config 5 in mode 3 default vs deterministic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_deterministic.py tests/test_gpu_zshift.py tests/test_gpu_z.py \
  > gpurun_out/r05n_tests.log 2>&1 || { tail -30 gpurun_out/r05n_tests.log; exit 1; }
tail -3 gpurun_out/r05n_tests.log
for m in 0 1 0 1; do
  ARPACK_HIP_DETERMINISTIC=$m timeout -k 10 200 python3 tools/c5_mode3.py > gpurun_out/r05n_c5_$m.json 2> gpurun_out/r05n_c5.err || { tail -5 gpurun_out/r05n_c5.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05n_c5_$m.json'));print('det=$m', {k:d[k] for k in ('cycles','opx','iters_per_s_incl_setup','bicgstab_iters_per_solve','ms_per_solve') if k in d}, d.get('steady_state',{}).get('cycles_per_s'), d['solver_roofline']['frac'])" | tee -a gpurun_out/r05n_c5.txt
done
