#!/bin/bash
# Client-side multi-tensor kernel variants: UNROLL -> fedscale_amd/variants/libfedagg_mt_u<UNROLL>.so
# (float4 per thread per chunk: 256 x 4 x UNROLL elements per workgroup); timed by tools/tune_prox.py
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for u in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DFA_TUNING=1 -DMT_UNROLL_N=$u \
    -o $ROOT/fedscale_amd/variants/libfedagg_mt_u$u.so $ROOT/fedscale_amd/csrc/client_update.hip \
    $ROOT/fedscale_amd/csrc/fedagg.hip &
done
wait
