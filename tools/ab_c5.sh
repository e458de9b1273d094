#!/bin/bash
# Interleaved A/B of whole libraries on config 5 as bench.py times it (q-FedAvg, chain launches unless AB_CHAIN=off,
# deferred gathers): FEDAGG_LIB=fedscale_amd/ab/libfedagg_<name>.so (built by tools/build_ab.sh), alternating,
# AB_REPS runs each.
#   bash tools/ab_c5.sh base mw        (AB_PARAMS=100000000 AB_STEPS=2: the one-GPU config 5; default: its shard of 8)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT
mkdir -p $ROOT/gpurun_out
for rep in $(seq 1 ${AB_REPS:-3}); do
  for name in "$@"; do
    out=$(FEDAGG_LIB=$ROOT/fedscale_amd/ab/libfedagg_$name.so timeout -k 10 240 python bench.py --config c5 --params ${AB_PARAMS:-12500000} --steps ${AB_STEPS:-3} --warmup 1 --cpu-seconds 0 --sustain 0 --mean-chain ${AB_CHAIN:-auto} --no-other-configs 2>$ROOT/gpurun_out/ab_${name}_err.log | grep '^{') || { echo "$name failed"; tail -5 $ROOT/gpurun_out/ab_${name}_err.log; exit 1; }
    python -c "import json,sys; d=json.loads(sys.argv[1]); print('$name', 'chain=${AB_CHAIN:-auto}', 'rep $rep', 'round_ms %.3f' % d['ms_per_step'], 'kernel_ms %.3f' % d['kernel_ms'], 'GB/s %.1f' % d['hbm_gbps'], 'passes', d['config'].get('streamed_passes'), 'launches', d['roofline']['launches_per_step'])" "$out"
  done
done
