#!/bin/bash
# PMC traffic of the fa_reduce workloads whose launch plan runs as column windows (FA_WINDOWS): the
# headline (1000 x 25M FedAvg), its 2-GPU bucket (12.5M), FedBuff and fused FedYoGi at 25M.  FETCH_SIZE and
# WRITE_SIZE in passes of their own; per-dispatch averages into profiles/pmc_traffic.json (other keys kept).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out
K=1000
for spec in "fedavg 25000000" "fedavg 12500032" "fedbuff 25000000" "fedyogi 25000000"; do
  set -- $spec
  pol=$1; P=$2
  ARGS="--policy $pol --params $P --steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmcw_${pol}_${P}_$c -o run -- python3 bench.py $ARGS > $OUT/pmcw_${pol}_${P}_$c.log 2>&1 || { tail -5 $OUT/pmcw_${pol}_${P}_$c.log; exit 1; }
  done
  case $pol in
    fedavg) ALG=$((4*K*P + 4*P)) ;;
    fedbuff) ALG=$((4*K*P + 4*P + 4*K)) ;;
    fedyogi) ALG=$((4*K*P + 24*P)) ;;
  esac
  W=$([ $pol = fedbuff ] && echo True || echo False)
  L=$(timeout -k 5 60 python -c "from fedscale_amd import kernels as kx; print(kx.reduce_launches($K, $P, weighted=$W))") || exit 1
  python tools/pmc_parse.py $OUT/pmcw_${pol}_${P}_FETCH_SIZE $OUT/pmcw_${pol}_${P}_WRITE_SIZE ${pol}_k${K}_p${P} $ALG k_reduce $L || exit 1
done
cp profiles/pmc_traffic.json $OUT/pmc_traffic_windows.json
