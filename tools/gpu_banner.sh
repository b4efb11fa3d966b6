# bench stdout carries exactly one JSON line with an RCCL communicator up;
# 2-rank host-transport rehearsal of the N > 1 bench path (both ranks on GPU 0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --rows 1250000 --steps 5 --warmup 2 --no-cpu-baseline --no-full-storage --no-ttc --force-dist > gpurun_out/r02g_fd.out 2> gpurun_out/r02g_fd.err || { tail -20 gpurun_out/r02g_fd.err; exit 1; }
wc -l gpurun_out/r02g_fd.out
python3 -c "import json; d=json.loads(open('gpurun_out/r02g_fd.out').read()); print('force-dist json ok', round(d['value'],1))"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --host-transport --rows 2000000 --steps 4 --warmup 1 > gpurun_out/r02g_ht.out 2> gpurun_out/r02g_ht.err || { tail -30 gpurun_out/r02g_ht.err; exit 1; }
wc -l gpurun_out/r02g_ht.out
python3 -c "import json; d=json.loads(open('gpurun_out/r02g_ht.out').read()); print('host-transport x2 json ok', round(d['value'],1), d['time_to_converge'], d['config']['parallelism'])"
