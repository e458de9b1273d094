#!/bin/bash
# Config 5's q-FedAvg phase 1 as the bench times it (chain launches, every pass), per library build
# (fedscale_amd/variants/libfedagg_qf2_*.so via FEDAGG_LIB), interleaved over REPS repetitions.
# usage: bash tools/qfed_lib_ab.sh [REPS] [PARAMS...]   (default params: 100000000 12500000)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
REPS=${1:-2}; shift
PS=${@:-100000000 12500000}
for r in $(seq $REPS); do
  for P in $PS; do
    for lib in fedscale_amd/variants/libfedagg_qf2_*.so; do
      out=$(FEDAGG_LIB=$ROOT/$lib timeout -k 10 240 python bench.py --config c5 --params $P --steps 2 --warmup 1 --cpu-seconds 0 --no-other-configs 2>/dev/null | grep '^{') || { echo "FAIL $lib $P"; exit 1; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"rep $r P=$P $(basename $lib .so): {d['kernel_ms']:9.2f} ms/round  {d['hbm_gbps']:7.0f} GB/s  launches {d['roofline']['launches_per_step']}\")"
    done
  done
done
