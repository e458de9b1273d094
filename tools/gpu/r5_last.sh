#!/bin/bash
# round 5, last tree: smoke(), the default line (auto warmup), a 2-rank gloo rehearsal of bench.py --gpus 2
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5zz_smoke.log 2>&1 || { tail -20 $O/r5zz_smoke.log; exit 1; }
grep smoke $O/r5zz_smoke.log
timeout -k 10 420 python -u bench.py > $O/r5zz_bench_n1.json 2> $O/r5zz_bench_n1.err || { tail -30 $O/r5zz_bench_n1.err; exit 1; }
echo bench ok
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 2 --steps 5 --dist-backend gloo --mem-fraction 0.25 --cpu-seconds 0 > $O/r5zz_rehearse_2.log 2>&1 || { tail -40 $O/r5zz_rehearse_2.log; exit 1; }
grep '^{' $O/r5zz_rehearse_2.log > $O/r5zz_bench_gloo_rehearsal_2.json
echo rehearsal ok
