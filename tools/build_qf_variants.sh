#!/bin/bash
# q-FedAvg phase-1 tuning variants: V,U,GRID,MIN_WAVES_PER_SIMD[,G[,BALANCE[,INFCHK[,PIPE]]]] -> fedscale_amd/variants/libfedagg_qf_*.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for spec in "$@"; do
  IFS=, read V U G W CG B I PP <<< "$spec"
  CG=${CG:-8}; B=${B:-1}; I=${I:-1}; PP=${PP:-0}
  out=$ROOT/fedscale_amd/variants/libfedagg_qf_v${V}_u${U}_g${G}_w${W}_c${CG}_b${B}_i${I}_p${PP}.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -DQF_V=$V -DQF_U=$U -DQF_GRID=$G -DQF_MINW=$W -DQF_G=$CG -DQF_BALANCE=$B -DQF_INFCHK=$I -DQF_PIPE=$PP \
    -o $out $ROOT/fedscale_amd/csrc/fedagg.hip &
done
wait
