#!/bin/bash
# Round-3 GPU sessions.  Every GPU step has its own time limit; the chain stops at the first failure.
#   test   pytest -m gpu + smoke
#   bench  default bench line (all configs)
#   c2     config 2 (100 x 1 M, two rotating input sets): rocprofv3 kernel trace + stats, FETCH_SIZE and
#          WRITE_SIZE passes (MI355X_MICROARCH.md's HBM recipe), per-launch traffic into profiles/pmc_traffic.json
#   c5     config 5's shard of 8 (10,000 x 12.5 M q-FedAvg, chain launches as the drop-in runs them): kernel
#          trace + stats, FETCH_SIZE / WRITE_SIZE, per-launch traffic into profiles/pmc_traffic.json
#   yogi   fused FedYoGi at 1000 x 25 M: VALU issue counters, FETCH_SIZE / WRITE_SIZE, kernel trace
#   head   headline kernel trace + stats (profiles/ summary of this round's library)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
for STAGE in "$@"; do
case $STAGE in
test)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r3_pytest_gpu.log 2>&1 || { tail -40 $OUT/r3_pytest_gpu.log; exit 1; }
  tail -2 $OUT/r3_pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r3_smoke.log 2>&1 || { tail -20 $OUT/r3_smoke.log; exit 1; }
  tail -1 $OUT/r3_smoke.log ;;
bench)
  timeout -k 10 600 python -u bench.py > $OUT/r3_bench.log 2>&1 || { tail -20 $OUT/r3_bench.log; exit 1; }
  grep '^{' $OUT/r3_bench.log | tail -1 | cut -c1-400 ;;
c2)
  ARGS="--config c2 --steps 200 --warmup 10 --cpu-seconds 0 --no-other-configs"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r3_c2_prof -o run -- python3 bench.py $ARGS > $OUT/r3_c2_prof.log 2>&1 || { tail -20 $OUT/r3_c2_prof.log; exit 1; }
  grep '^{' $OUT/r3_c2_prof.log | cut -c1-300
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/r3_c2_$c -o run -- python3 bench.py --config c2 --steps 20 --warmup 2 --cpu-seconds 0 --no-other-configs > $OUT/r3_c2_$c.log 2>&1 || { tail -5 $OUT/r3_c2_$c.log; exit 1; }
  done
  L=$(timeout -k 5 60 python -c "from fedscale_amd import kernels as kx; print(kx.reduce_launches(100, 1000000))") || exit 1
  python tools/pmc_parse.py $OUT/r3_c2_FETCH_SIZE $OUT/r3_c2_WRITE_SIZE fedavg_k100_p1000000 $((4*100*1000000 + 4*1000000)) k_reduce $L || exit 1 ;;
c5)
  ARGS="--config c5 --params 12500000 --steps 2 --warmup 1 --cpu-seconds 0 --no-other-configs"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r3_c5_prof -o run -- python3 bench.py $ARGS > $OUT/r3_c5_prof.log 2>&1 || { tail -20 $OUT/r3_c5_prof.log; exit 1; }
  grep '^{' $OUT/r3_c5_prof.log | cut -c1-300
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/r3_c5_$c -o run -- python3 bench.py --config c5 --params 12500000 --steps 1 --warmup 0 --cpu-seconds 0 --no-other-configs > $OUT/r3_c5_$c.log 2>&1 || { tail -5 $OUT/r3_c5_$c.log; exit 1; }
  done
  # per-launch algorithmic bytes and launches per step from the traced run's own bench line
  AL=$(grep '^{' $OUT/r3_c5_prof.log | tail -1 | python -c "import json,sys; r=json.loads(sys.stdin.read())['roofline']; print(int(r['alg_bytes_per_launch'] * r['launches_per_step']), 'k_qfed_accum', r['launches_per_step'])") || exit 1
  python tools/pmc_parse.py $OUT/r3_c5_FETCH_SIZE $OUT/r3_c5_WRITE_SIZE qfedavg_k10000_p12500000 $AL > $OUT/r3_c5_pmc.json || exit 1
  cat $OUT/r3_c5_pmc.json ;;
yogi)
  ARGS="--policy fedyogi --steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs"
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/r3_yogi_valu -o run -- python3 bench.py $ARGS > $OUT/r3_yogi_valu.log 2>&1 || { tail -5 $OUT/r3_yogi_valu.log; exit 1; }
  python tools/pmc_valu_parse.py $OUT/r3_yogi_valu k_reduce 25000000 > $OUT/r3_yogi_valu.json || exit 1
  cat $OUT/r3_yogi_valu.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r3_yogi_prof -o run -- python3 bench.py --policy fedyogi --steps 10 --warmup 2 --cpu-seconds 0 --no-other-configs > $OUT/r3_yogi_prof.log 2>&1 || { tail -20 $OUT/r3_yogi_prof.log; exit 1; }
  grep '^{' $OUT/r3_yogi_prof.log | cut -c1-300 ;;
head)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r3_head_prof -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-other-configs > $OUT/r3_head_prof.log 2>&1 || { tail -20 $OUT/r3_head_prof.log; exit 1; }
  grep '^{' $OUT/r3_head_prof.log | cut -c1-300 ;;
headpmc)  # headline FETCH_SIZE / WRITE_SIZE passes (one counter block each), per-launch traffic into profiles/pmc_traffic.json
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/r3_head_$c -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs > $OUT/r3_head_$c.log 2>&1 || { tail -5 $OUT/r3_head_$c.log; exit 1; }
  done
  L=$(timeout -k 5 60 python -c "from fedscale_amd import kernels as kx; print(kx.reduce_launches(1000, 25000000))") || exit 1
  python tools/pmc_parse.py $OUT/r3_head_FETCH_SIZE $OUT/r3_head_WRITE_SIZE fedavg_k1000_p25000000 $((4*1000*25000000 + 4*25000000)) k_reduce $L || exit 1 ;;
dist)  # gloo rehearsals (ranks share the one GPU): per-rank kernel times on the N > 1 lines
  for n in 2 4; do
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 5 --warmup 1 --dist-backend gloo --mem-fraction 0.15 --no-other-configs > $OUT/r3_dist$n.log 2>&1 || { tail -30 $OUT/r3_dist$n.log; exit 1; }
    grep '^{' $OUT/r3_dist$n.log | cut -c1-200
  done ;;
*) echo "unknown stage $STAGE"; exit 2 ;;
esac
done
