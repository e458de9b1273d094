# round 5, last tree: GPU suite, smoke(), the default line, and 2- / 8-rank gloo
# rehearsals of bench.py --gpus N
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r5w_pytest_gpu.log 2>&1 || { tail -30 $O/r5w_pytest_gpu.log; exit 1; }
tail -1 $O/r5w_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5w_smoke.log 2>&1 || { tail -20 $O/r5w_smoke.log; exit 1; }
cat $O/r5w_smoke.log | grep smoke
timeout -k 10 420 python -u bench.py > $O/r5w_bench_n1.json 2> $O/r5w_bench_n1.err || { tail -30 $O/r5w_bench_n1.err; exit 1; }
echo bench ok
for N in 2 8; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29540 + N)) bench.py --gpus $N --steps 5 --warmup 2 --dist-backend gloo --mem-fraction $(python -c "print(round(0.5 / $N, 3))") --cpu-seconds 0 > $O/r5w_rehearse_$N.log 2>&1 || { tail -40 $O/r5w_rehearse_$N.log; exit 1; }
  grep '^{' $O/r5w_rehearse_$N.log > $O/r5w_bench_gloo_rehearsal_$N.json
done
echo rehearsals ok
