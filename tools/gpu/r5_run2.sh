# round 5: GPU suite, the default N=1 bench line (with the sustained leg and card telemetry), and the 8-rank gloo
# rehearsal of bench.py --gpus 8 on the one card (the in-process leg at 8 parts)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r5_pytest_gpu2.log 2>&1 || { tail -30 $O/r5_pytest_gpu2.log; exit 1; }
tail -2 $O/r5_pytest_gpu2.log
timeout -k 10 420 python -u bench.py > $O/r5_bench_n1.json 2> $O/r5_bench_n1.err || { tail -30 $O/r5_bench_n1.err; exit 1; }
echo bench ok
N=8
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus $N --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.06 --cpu-seconds 0 > $O/r5_rehearse_8.log 2>&1 || { tail -40 $O/r5_rehearse_8.log; exit 1; }
grep '^{' $O/r5_rehearse_8.log > $O/r5_bench_gloo_rehearsal_8.json
echo rehearsal ok
