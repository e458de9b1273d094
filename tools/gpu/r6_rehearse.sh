#!/bin/bash
# round 6: the final bench.py — the driver's N = 1 scaling invocation (torch.distributed.run, one process), then
# bench.py --gpus 2 / 8 as gloo ranks on the one card
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r6r_torchrun_n1.log 2>&1 || { tail -40 $O/r6r_torchrun_n1.log; exit 1; }
grep '^{' $O/r6r_torchrun_n1.log > $O/r6r_bench_torchrun_n1.json
echo torchrun ok
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.2 --cpu-seconds 3 > $O/r6r_rehearse_2.log 2>&1 || { tail -40 $O/r6r_rehearse_2.log; exit 1; }
grep '^{' $O/r6r_rehearse_2.log > $O/r6r_bench_gloo_rehearsal_2.json
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.06 --cpu-seconds 3 > $O/r6r_rehearse_8.log 2>&1 || { tail -40 $O/r6r_rehearse_8.log; exit 1; }
grep '^{' $O/r6r_rehearse_8.log > $O/r6r_bench_gloo_rehearsal_8.json
echo rehearsals ok
