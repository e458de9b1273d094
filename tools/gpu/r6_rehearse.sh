#!/bin/bash
# round 6: the final bench.py — the default N = 1 line, then bench.py --gpus 2 / 8 as gloo ranks on the one card
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py > $O/r6h_bench_n1.json 2> $O/r6h_bench_n1.err || { tail -30 $O/r6h_bench_n1.err; exit 1; }
echo bench ok
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.2 --cpu-seconds 3 > $O/r6h_rehearse_2.log 2>&1 || { tail -40 $O/r6h_rehearse_2.log; exit 1; }
grep '^{' $O/r6h_rehearse_2.log > $O/r6h_bench_gloo_rehearsal_2.json
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.06 --cpu-seconds 3 > $O/r6h_rehearse_8.log 2>&1 || { tail -40 $O/r6h_rehearse_8.log; exit 1; }
grep '^{' $O/r6h_rehearse_8.log > $O/r6h_bench_gloo_rehearsal_8.json
echo rehearsals ok
