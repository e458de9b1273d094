#!/bin/bash
# Library builds with arbitrary compile-time knobs, for tools/tune_qfed2.py / tools/qfed_lib_ab.sh:
#   bash tools/build_qf_defs.sh NAME="-DQF_CHAIN_V=16 -DQF_WIN_ROUNDS=2" NAME2="" ...
# -> fedscale_amd/variants/libfedagg_qf2_NAME.so (an empty definition list is the production build)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for spec in "$@"; do
  name=${spec%%=*}
  defs=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DFA_TUNING=1 $defs \
    -o $ROOT/fedscale_amd/variants/libfedagg_qf2_$name.so $ROOT/fedscale_amd/csrc/fedagg.hip \
    $ROOT/fedscale_amd/csrc/client_update.hip $ROOT/fedscale_amd/csrc/ingress_host.cpp $ROOT/fedscale_amd/csrc/ingress_dma.cpp \
    $ROOT/fedscale_amd/csrc/rccl_comm.cpp &
done
wait
ls $ROOT/fedscale_amd/variants
