#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
STAGE=${1:-all}
run() { echo "== $*" ; }
if [[ $STAGE == all || $STAGE == test ]]; then
  run tests
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  run bench
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  run rocprof
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-other-configs > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  tail -1 $OUT/prof.log
  find $OUT/prof -name "*kernel_stats.csv" | head -3
fi
if [[ $STAGE == pmc ]]; then
  export TMPDIR=/tmp
  ARGS="--steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs"
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py $ARGS > $OUT/pmc_fetch.log 2>&1 || { tail -20 $OUT/pmc_fetch.log; exit 1; }
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py $ARGS > $OUT/pmc_write.log 2>&1 || { tail -20 $OUT/pmc_write.log; exit 1; }
  rm -f profiles/pmc_traffic.json
  python tools/pmc_parse.py $OUT/pmc_fetch $OUT/pmc_write fedavg_k1000_p25000000 $((4*1000*25000000 + 4*25000000)) && cp profiles/pmc_traffic.json $OUT/
fi
if [[ $STAGE == pmcpol ]]; then  # the other server steps' dominant kernels (bench --policy ...)
  export TMPDIR=/tmp
  K=1000; P=25000000
  rm -f profiles/pmc_traffic.json
  for pol in fedbuff fedyogi qfedavg; do
    ARGS="--policy $pol --steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs"
    timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$pol -o run -- python3 $ROOT/bench.py $ARGS > $OUT/pmc_fetch_$pol.log 2>&1 || { tail -20 $OUT/pmc_fetch_$pol.log; exit 1; }
    timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$pol -o run -- python3 $ROOT/bench.py $ARGS > $OUT/pmc_write_$pol.log 2>&1 || { tail -20 $OUT/pmc_write_$pol.log; exit 1; }
    case $pol in
      fedbuff) ALG=$((4*K*P + 4*P + 4*K)); KERN=k_reduce ;;
      fedyogi) ALG=$((4*K*P + 24*P)); KERN=k_reduce ;;
      qfedavg) ALG=$((4*K*P + 8*P + 8*K)); KERN=k_qfed_accum ;;
    esac
    python tools/pmc_parse.py $OUT/pmc_fetch_$pol $OUT/pmc_write_$pol ${pol}_k${K}_p${P} $ALG $KERN || exit 1
  done
  cp profiles/pmc_traffic.json $OUT/pmc_traffic_policies.json
fi
if [[ $STAGE == tune ]]; then
  timeout -k 10 300 python tools/hbm_ceiling.py 64 > $OUT/ceiling.log 2>&1 || { tail -20 $OUT/ceiling.log; exit 1; }
  cat $OUT/ceiling.log
  timeout -k 10 900 python tools/tune_reduce.py 1000 25000000 5 > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
  cat $OUT/tune.log
  timeout -k 10 600 python tools/tune_reduce.py 100 1000000 7 > $OUT/tune_c2.log 2>&1 || { tail -20 $OUT/tune_c2.log; exit 1; }
  cat $OUT/tune_c2.log
fi
if [[ $STAGE == sweep ]]; then
  timeout -k 10 1000 python tools/tune_reduce.py sweep ${SWEEP:-1000:25000000,1000:11191242,1000:12500000,400:50000000,1000:4000000,100:1000000} ${SWR:-3} > $OUT/sweep.log 2>&1 || { tail -20 $OUT/sweep.log; exit 1; }
  cat $OUT/sweep.log
fi
if [[ $STAGE == dist ]]; then
  timeout -k 10 900 python -m pytest tests/test_distributed.py -m gpu -x -q > $OUT/pytest_dist.log 2>&1 || { tail -40 $OUT/pytest_dist.log; exit 1; }
  tail -3 $OUT/pytest_dist.log
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --clients 100 --params 4000000 --dist-backend gloo --mem-fraction 0.3 > $OUT/bench_dist2.log 2>&1 || { tail -30 $OUT/bench_dist2.log; exit 1; }
  grep '^{' $OUT/bench_dist2.log
  for pol in fedavg fedyogi qfedavg; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 1 --clients 100 --params 4000000 --dist-backend gloo --shard clients --policy $pol > $OUT/bench_dist2_clients_$pol.log 2>&1 || { tail -30 $OUT/bench_dist2_clients_$pol.log; exit 1; }
    grep '^{' $OUT/bench_dist2_clients_$pol.log
  done
  timeout -k 10 300 python bench.py --shard clients --steps 5 --warmup 1 --cpu-seconds 0 --no-other-configs > $OUT/bench_clients_n1.log 2>&1 || { tail -30 $OUT/bench_clients_n1.log; exit 1; }
  grep '^{' $OUT/bench_clients_n1.log
fi
if [[ $STAGE == ingress ]]; then
  timeout -k 10 600 python tools/ingress_bench.py 200 3 resnet18 ${WORKERS:-1,4,8,16} > $OUT/ingress.log 2>&1 || { tail -30 $OUT/ingress.log; exit 1; }
  grep '^{' $OUT/ingress.log
fi
if [[ $STAGE == policies ]]; then
  for pol in ${POLS:-fedbuff fedyogi qfedavg}; do
    timeout -k 10 300 python bench.py --policy $pol --steps 10 --cpu-seconds 0 > $OUT/bench_$pol.log 2>&1 || { tail -20 $OUT/bench_$pol.log; exit 1; }
    grep '^{' $OUT/bench_$pol.log
  done
fi
if [[ $STAGE == tuneqf ]]; then
  for P in ${QFP:-25000000}; do
    timeout -k 10 600 python tools/tune_qfed.py ${QFK:-1000} $P ${QFR:-3} > $OUT/tune_qf_$P.log 2>&1 || { tail -20 $OUT/tune_qf_$P.log; exit 1; }
    cat $OUT/tune_qf_$P.log
  done
fi
