# Padded V columns: full GPU suite, smoke, then config 4 (n = 215^3, odd) with
# the device V's ldv padded to 128 B (default) and unpadded, alternating.
set -o pipefail
TAG=${1:-ldv}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
for p in 1 0 1 0; do
  ARPACK_HIP_LDV_PAD=$p timeout -k 10 200 python3 tools/bench_configs.py C4 > gpurun_out/${TAG}_c4_pad$p.json 2>>gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_c4_pad$p.json'))['C4_dsaupd_lap3d_9.94e6']['full_storage'];print('pad=$p', round(d['iters_per_s'],2), {k:(round(v['ms']/max(v['launches'],1)*1e3,1), round(v['gbs'] or 0)) for k,v in d['roofline']['kernels'].items()})" | tee -a gpurun_out/${TAG}_c4_summary.txt
done
