#!/bin/bash
# round 6, the library the round ends with: the GPU suite + smoke, the default N = 1 line, rocprofv3 kernel stats of
# the headline command, its PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs), bench.py under torch.distributed.run
# with one process (the driver's N = 1 scaling invocation), and the 2- and 8-rank gloo rehearsals
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6f_pytest_gpu.log 2>&1 || { tail -40 $O/r6f_pytest_gpu.log; exit 1; }
tail -1 $O/r6f_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r6f_smoke.log 2>&1 || { tail -20 $O/r6f_smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/r6f_bench_n1.json 2> $O/r6f_bench_n1.err || { tail -30 $O/r6f_bench_n1.err; exit 1; }
echo bench ok
H="bench.py --no-other-configs --cpu-seconds 0 --sustain 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r6f_head_trace -o head --output-format csv -- python3 $H > $O/r6f_head_under_rocprof.json 2> $O/r6f_head_trace.err || { tail -20 $O/r6f_head_trace.err; exit 1; }
echo trace ok
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/r6f_pmc_fetch -o pmc --output-format csv -- python3 $H --steps 3 --warmup 1 > $O/r6f_pmc_fetch.json 2> $O/r6f_pmc_fetch.err || { tail -20 $O/r6f_pmc_fetch.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/r6f_pmc_write -o pmc --output-format csv -- python3 $H --steps 3 --warmup 1 > $O/r6f_pmc_write.json 2> $O/r6f_pmc_write.err || { tail -20 $O/r6f_pmc_write.err; exit 1; }
echo pmc ok
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > $O/r6f_torchrun_n1.log 2>&1 || { tail -40 $O/r6f_torchrun_n1.log; exit 1; }
grep '^{' $O/r6f_torchrun_n1.log > $O/r6f_bench_torchrun_n1.json
echo torchrun ok
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.2 --cpu-seconds 3 > $O/r6f_rehearse_2.log 2>&1 || { tail -40 $O/r6f_rehearse_2.log; exit 1; }
grep '^{' $O/r6f_rehearse_2.log > $O/r6f_bench_gloo_rehearsal_2.json
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 8 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.06 --cpu-seconds 3 > $O/r6f_rehearse_8.log 2>&1 || { tail -40 $O/r6f_rehearse_8.log; exit 1; }
grep '^{' $O/r6f_rehearse_8.log > $O/r6f_bench_gloo_rehearsal_8.json
echo rehearsals ok
