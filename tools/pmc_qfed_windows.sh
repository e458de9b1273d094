#!/bin/bash
# PMC traffic of q-FedAvg phase 1 with its column-window launches (bench.py --policy qfedavg, 1000 x 25M):
# FETCH_SIZE and WRITE_SIZE in passes of their own; per-dispatch averages into profiles/pmc_traffic.json.
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out
K=1000; P=25000000
ARGS="--policy qfedavg --steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmcq_$c -o run -- python3 bench.py $ARGS > $OUT/pmcq_$c.log 2>&1 || { tail -5 $OUT/pmcq_$c.log; exit 1; }
done
L=$(timeout -k 5 60 python -c "from fedscale_amd import kernels as kx; print(kx.qfed_launches($P, $P))") || exit 1
python tools/pmc_parse.py $OUT/pmcq_FETCH_SIZE $OUT/pmcq_WRITE_SIZE qfedavg_k${K}_p${P} $((4*K*P + 8*P + 8*K)) k_qfed_accum $L || exit 1
cp profiles/pmc_traffic.json $OUT/pmc_traffic_qfed_windows.json
