#!/bin/bash
# What outlives bench.py (VERDICT r04 hygiene item): processes before and after
# a bench run with the CPU baseline leg, and the plain-command N-rank rehearsal.
set -o pipefail
TAG=${1:-hyg}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ps -eo pid,ppid,pgid,sid,stat,etime,args > gpurun_out/${TAG}_ps_before.txt
timeout -k 10 300 python3 bench.py --rows 1000000 --steps 4 --warmup 1 --no-full-storage > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
sleep 3
ps -eo pid,ppid,pgid,sid,stat,etime,args > gpurun_out/${TAG}_ps_after.txt
timeout -k 10 300 python3 bench.py --gpus 2 --host-transport --rows 2000000 --steps 4 > gpurun_out/${TAG}_two_ranks.json 2> gpurun_out/${TAG}_two_ranks.err || exit $?
sleep 3
ps -eo pid,ppid,pgid,sid,stat,etime,args > gpurun_out/${TAG}_ps_after2.txt
python3 bench.py --gpus 2 > gpurun_out/${TAG}_no_gpus.out 2>&1; echo "rc=$?" >> gpurun_out/${TAG}_no_gpus.out
diff <(awk '{print $NF}' gpurun_out/${TAG}_ps_before.txt | sort) <(awk '{print $NF}' gpurun_out/${TAG}_ps_after.txt | sort); true
