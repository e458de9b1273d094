#!/bin/bash
# q-FedAvg phase-1 kernel variants: KERNEL,CHAIN_KERNEL,V,WAVES[,GRID[,GLDS[,EMAX[,PART[,WIDE_BYTES]]]]] -> fedscale_amd/variants/libfedagg_qf2_*.so
# (1 = the 1-wave/SIMD register design, 2 = the LDS-`last` 2-pass design; KERNEL serves launches without the
#  fused FedAvg chain, CHAIN_KERNEL those with it; V / WAVES / GRID apply to design 2)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for spec in "$@"; do
  IFS=, read KK CK V W G GL EM PT WB <<< "$spec"
  G=${G:-256}; GL=${GL:-0}; EM=${EM:-1}; PT=${PT:-4}; WB=${WB:-2147483648}
  out=$ROOT/fedscale_amd/variants/libfedagg_qf2_k${KK}_c${CK}_v${V}_w${W}_g${G}_l${GL}_e${EM}_p${PT}_wb${WB}.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DFA_TUNING=1 \
    -DQF_KERNEL=$KK -DQF_CHAIN_KERNEL=$CK -DQF2_V=$V -DQF2_WAVES=$W -DQF2_GRID=$G -DQF_PLAIN_GLDS=$GL -DQF_CHAIN_GLDS=$GL -DQF_EMAX=$EM -DQF_PART=$PT -DQF_WIDE_BYTES=${WB}LL \
    -o $out $ROOT/fedscale_amd/csrc/fedagg.hip $ROOT/fedscale_amd/csrc/client_update.hip \
    $ROOT/fedscale_amd/csrc/ingress_host.cpp $ROOT/fedscale_amd/csrc/ingress_dma.cpp $ROOT/fedscale_amd/csrc/rccl_comm.cpp &
done
wait
