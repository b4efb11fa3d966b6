set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for fd in "" "--force-dist"; do
    for rows in 10000000 1250000; do
      st=20; [ $rows = 1250000 ] && st=100
      out=gpurun_out/r04r_${rep}_${rows}${fd:+_fd}.json
      timeout -k 10 200 python3 bench.py --steps $st --warmup 5 --no-cpu-baseline --no-full-storage --no-ttc --rows $rows $fd > $out 2>gpurun_out/r04r.err || { tail -5 gpurun_out/r04r.err; exit 1; }
      python3 -c "import json;d=json.load(open('$out'));print('$rep', '$rows', '${fd:-plain}', round(d['value'],2), {k:(v['launches'], round(v['ms']/max(v['launches'],1)*1e3,1)) for k,v in d['kernels'].items() if v['launches']})"
    done
  done
done
