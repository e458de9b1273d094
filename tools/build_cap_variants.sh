#!/bin/bash
# fa_reduce multi-round capped-plan variants: SW_MAX[,CAP_PCT] -> fedscale_amd/variants/libfedagg_cap_sw<S>_c<C>.so
# (widest tile of the R-rounds plan, grid cap in % of the CUs); timed by tools/tune_reduce.py
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for spec in "$@"; do
  IFS=, read S C <<< "$spec"
  C=${C:-75}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DFA_TUNING=1 \
    -DFA_CAP_SW_MAX=$S -DFA_GRID_CAP_PCT=$C \
    -o $ROOT/fedscale_amd/variants/libfedagg_cap_sw${S}_c${C}.so $ROOT/fedscale_amd/csrc/fedagg.hip &
done
wait
