# Same-box A/B of the bench warmup length in fresh processes (W=2, the default, vs 30):
# with W >= the solve's convergence count the timed cycles come from a fresh solve.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for i in 1 2 3; do
 for w in 2 30; do
  timeout -k 10 200 python3 bench.py --warmup $w --no-cpu-baseline --no-ttc --no-full-storage --no-profile > gpurun_out/wu_$w.json 2>gpurun_out/wu.err || { tail -5 gpurun_out/wu.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/wu_$w.json'));print('W=$w', round(d['value'],2))"
 done
done
