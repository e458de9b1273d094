# round 5, final library: GPU suite, the default N=1 line, rocprofv3 kernel stats + PMC (FETCH_SIZE / WRITE_SIZE in
# separate passes) of the headline command, and the 8-rank gloo rehearsal of bench.py --gpus 8
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r5f_pytest_gpu.log 2>&1 || { tail -30 $O/r5f_pytest_gpu.log; exit 1; }
tail -1 $O/r5f_pytest_gpu.log
timeout -k 10 420 python -u bench.py > $O/r5f_bench_n1.json 2> $O/r5f_bench_n1.err || { tail -30 $O/r5f_bench_n1.err; exit 1; }
echo bench ok
H="bench.py --no-other-configs --cpu-seconds 0 --sustain 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r5f_head_trace -o head --output-format csv -- python3 $H > $O/r5f_head_under_rocprof.json 2> $O/r5f_head_trace.err || { tail -20 $O/r5f_head_trace.err; exit 1; }
echo trace ok
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/r5f_pmc_fetch -o pmc --output-format csv -- python3 $H --steps 3 --warmup 1 > $O/r5f_pmc_fetch.json 2> $O/r5f_pmc_fetch.err || { tail -20 $O/r5f_pmc_fetch.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/r5f_pmc_write -o pmc --output-format csv -- python3 $H --steps 3 --warmup 1 > $O/r5f_pmc_write.json 2> $O/r5f_pmc_write.err || { tail -20 $O/r5f_pmc_write.err; exit 1; }
echo pmc ok
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.06 --cpu-seconds 0 > $O/r5f_rehearse_8.log 2>&1 || { tail -40 $O/r5f_rehearse_8.log; exit 1; }
grep '^{' $O/r5f_rehearse_8.log > $O/r5f_bench_gloo_rehearsal_8.json
echo rehearsal ok
