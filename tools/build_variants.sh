#!/bin/bash
# Compile fa_reduce tuning variants (V float4/lane, U clients in flight, NT loads) into fedscale_amd/variants/.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for spec in "$@"; do
  IFS=, read V U NT W <<< "$spec"
  W=${W:-4}
  out=$ROOT/fedscale_amd/variants/libfedagg_v${V}_u${U}_nt${NT}_w${W}.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -DFA_RED_V=$V -DFA_RED_U=$U -DFA_RED_NT=$NT -DFA_RED_WAVES=$W -o $out $ROOT/fedscale_amd/csrc/fedagg.hip &
done
wait
ls $ROOT/fedscale_amd/variants
