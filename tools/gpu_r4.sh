#!/bin/bash
# Round-4 GPU sessions.  Every GPU step has its own time limit; the chain stops at the first failure.
#   test     pytest -m gpu + smoke
#   tune5    q-FedAvg chain-grid variants (fedscale_amd/variants, tools/build_qf_defs.sh), interleaved:
#            config 5's shard chunk (1024 x 12.5 M, first and later passes) and 1000 x 25 M
#   reg      N-GPU ingress: gather into a pinned row vs hipHostRegister of the payload (tools/register_probe.py)
#   sreg     the same through ShardedModelAdapter (RegisteredUpload vs the pinned-row gather), 1/2/4 parts
#   bench    default bench line (all configs)
#   c4       config 4 as the drop-in runs it (mean, then k_yogi_step): kernel trace + stats
#   c5       config 5's shard of 8: kernel trace + stats, FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md recipe)
#   head     headline kernel trace + stats
#   c4pmc / headpmc  FETCH_SIZE / WRITE_SIZE passes of config 4's unfused round / the headline
#   rehearse 2- and 4-rank gloo rehearsals of bench.py --gpus N on the one card (plumbing of the N-GPU fields)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
T=${TAG:-r4}
for STAGE in "$@"; do
case $STAGE in
test)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/${T}_pytest_gpu.log 2>&1 || { tail -40 $OUT/${T}_pytest_gpu.log; exit 1; }
  tail -2 $OUT/${T}_pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || { tail -20 $OUT/${T}_smoke.log; exit 1; }
  tail -1 $OUT/${T}_smoke.log ;;
tune5)
  timeout -k 10 300 python -u tools/tune_qfed2.py 1024 12500000 5 > $OUT/${T}_tune5_first.log 2>&1 || { tail -20 $OUT/${T}_tune5_first.log; exit 1; }
  cat $OUT/${T}_tune5_first.log
  timeout -k 10 300 python -u tools/tune_qfed2.py 1024 12500000 5 acc > $OUT/${T}_tune5_acc.log 2>&1 || { tail -20 $OUT/${T}_tune5_acc.log; exit 1; }
  cat $OUT/${T}_tune5_acc.log
  timeout -k 10 300 python -u tools/tune_qfed2.py 1000 25000000 3 > $OUT/${T}_tune5_25m.log 2>&1 || { tail -20 $OUT/${T}_tune5_25m.log; exit 1; }
  cat $OUT/${T}_tune5_25m.log ;;
reg)
  for L in p25m resnet18; do
    timeout -k 10 300 python -u tools/register_probe.py $L 1,2,4 16 > $OUT/${T}_register_$L.log 2>&1 || { tail -20 $OUT/${T}_register_$L.log; exit 1; }
    cat $OUT/${T}_register_$L.log
  done ;;
sreg)
  for L in p25m resnet18; do
    timeout -k 10 400 python -u tools/sharded_ingress_bench.py 24 3 $L 1,2,4 payload > $OUT/${T}_sharded_ingress_$L.log 2>&1 || { tail -20 $OUT/${T}_sharded_ingress_$L.log; exit 1; }
    grep '^{' $OUT/${T}_sharded_ingress_$L.log
  done ;;
bench)
  timeout -k 10 700 python -u bench.py > $OUT/${T}_bench.log 2>&1 || { tail -20 $OUT/${T}_bench.log; exit 1; }
  grep '^{' $OUT/${T}_bench.log | tail -1 | cut -c1-600 ;;
c4)
  ARGS="--config c4 --steps 10 --warmup 2 --cpu-seconds 0 --no-other-configs"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${T}_c4_prof -o run -- python3 bench.py $ARGS > $OUT/${T}_c4_prof.log 2>&1 || { tail -20 $OUT/${T}_c4_prof.log; exit 1; }
  grep '^{' $OUT/${T}_c4_prof.log | cut -c1-900 ;;
c5)
  ARGS="--config c5 --params 12500000 --steps 2 --warmup 1 --cpu-seconds 0 --no-other-configs"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${T}_c5_prof -o run -- python3 bench.py $ARGS > $OUT/${T}_c5_prof.log 2>&1 || { tail -20 $OUT/${T}_c5_prof.log; exit 1; }
  grep '^{' $OUT/${T}_c5_prof.log | cut -c1-400
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/${T}_c5_$c -o run -- python3 bench.py $ARGS > $OUT/${T}_c5_$c.log 2>&1 || { tail -5 $OUT/${T}_c5_$c.log; exit 1; }
  done ;;
c4pmc|headpmc)
  # FETCH_SIZE / WRITE_SIZE of config 4's unfused round (k_reduce x 4 + k_yogi_step) or the headline, one pass each
  [ $STAGE = c4pmc ] && ARGS="--config c4 --steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs" || ARGS="--steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/${T}_${STAGE}_$c -o run -- python3 bench.py $ARGS > $OUT/${T}_${STAGE}_$c.log 2>&1 || { tail -5 $OUT/${T}_${STAGE}_$c.log; exit 1; }
  done
  grep '^{' $OUT/${T}_${STAGE}_FETCH_SIZE.log | cut -c1-300 ;;
head)
  ARGS="--steps 12 --warmup 3 --cpu-seconds 0 --no-other-configs"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${T}_head_prof -o run -- python3 bench.py $ARGS > $OUT/${T}_head_prof.log 2>&1 || { tail -20 $OUT/${T}_head_prof.log; exit 1; }
  grep '^{' $OUT/${T}_head_prof.log | cut -c1-400 ;;
rehearse)
  for N in 2 4; do
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 1 --dist-backend gloo --mem-fraction $(python -c "print(round(0.5 / $N, 3))") --cpu-seconds 0 > $OUT/${T}_rehearse_$N.log 2>&1 || { tail -30 $OUT/${T}_rehearse_$N.log; exit 1; }
    grep '^{' $OUT/${T}_rehearse_$N.log | tail -1 | cut -c1-1500
  done ;;
*)
  echo "unknown stage $STAGE"; exit 2 ;;
esac
done
