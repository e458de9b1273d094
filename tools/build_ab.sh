#!/bin/bash
# Whole-library A/B variants for tools/ab_c5.sh: fedscale_amd/ab/libfedagg_<name>.so from the current sources with
# extra -D flags.  Rebuild after any change to the ABI (bench.py loads every symbol of the header's table).
#   bash tools/build_ab.sh base ""  maxk2048 "-DQF_MAXK=2048"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/fedscale_amd/csrc
mkdir -p $ROOT/fedscale_amd/ab
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wall $defs \
    -o $ROOT/fedscale_amd/ab/libfedagg_$name.so $C/fedagg.hip $C/client_update.hip $C/ingress_host.cpp \
    $C/ingress_dma.cpp $C/rccl_comm.cpp
  echo "built ab/libfedagg_$name.so ($defs)"
done
