#!/bin/bash
# HeteroFL prefix-box kernel variants: J,U,DPREFETCH -> fedscale_amd/variants/libfedagg_hb_j<J>_u<U>_dp<D>.so
# (J float4 groups per thread in FLAT mode, U clients in flight, D = next-descriptor prefetch); timed by
# tools/tune_heterofl.py
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for spec in "$@"; do
  IFS=, read J U D <<< "$spec"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DFA_TUNING=1 \
    -DHB_FLAT_J=$J -DHB_FLAT_U=$U -DHB_DPREFETCH=$D \
    -o $ROOT/fedscale_amd/variants/libfedagg_hb_j${J}_u${U}_dp${D}_.so $ROOT/fedscale_amd/csrc/fedagg.hip &
done
wait
