#!/bin/bash
# Round-5 deterministic symmetric SpMV (k_csr_ssell_det): its GPU tests, a
# same-box bench A/B against the default kernel, and the TTC repeat (bitwise).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_deterministic.py tests/test_gpu_symspmv_handoff.py \
  "tests/test_gpu_dist.py::test_symmetric_storage_deterministic_ranks" \
  > gpurun_out/r05l_tests.log 2>&1 || { tail -30 gpurun_out/r05l_tests.log; exit 1; }
tail -3 gpurun_out/r05l_tests.log
for m in def det def det; do
  f=""; [ $m = det ] && f="--deterministic"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ttc $f > gpurun_out/r05l_ab_$m.json 2> gpurun_out/r05l_ab.err || { tail -5 gpurun_out/r05l_ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05l_ab_$m.json'));print('$m', round(d['value'],2), 'full', round(d['full_storage']['value'],2), d['config']['bitwise_reproducible'], {k:(v['launches'], round(v['ms']/max(v['launches'],1)*1e3,1)) for k,v in d['kernels'].items() if v['launches']})" | tee -a gpurun_out/r05l_ab.txt
done
timeout -k 10 300 python3 tools/ttc_repeat.py --repeats 3 > gpurun_out/r05l_ttc.json 2> gpurun_out/r05l_ttc.err || { tail -5 gpurun_out/r05l_ttc.err; exit 1; }
cat gpurun_out/r05l_ttc.err
