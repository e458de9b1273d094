#!/bin/bash
# Compile fa_reduce tuning variants into fedscale_amd/variants/.  spec: V,U,NT[,WAVES[,GRID]]
#   V float4 per lane, U clients in flight, NT non-temporal loads, WAVES per workgroup, GRID > 0: a capped
#   grid of GRID workgroups each walking an equal number of tiles (0: one workgroup per tile), PIPE 1 the
#   software-pipelined client groups (FA_PIPE).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/variants
cd /tmp
for spec in "$@"; do
  IFS=, read V U NT W G PP <<< "$spec"
  W=${W:-4}
  G=${G:-0}
  PP=${PP:-0}
  out=$ROOT/fedscale_amd/variants/libfedagg_v${V}_u${U}_nt${NT}_w${W}_g${G}_p${PP}.so
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DFA_TUNING=1 \
    -DFA_RED_V=$V -DFA_RED_U=$U -DFA_RED_NT=$NT -DFA_RED_WAVES=$W -DFA_RED_GRID=$G -DFA_PIPE=$PP \
    -o $out $ROOT/fedscale_amd/csrc/fedagg.hip &
done
wait
ls $ROOT/fedscale_amd/variants
