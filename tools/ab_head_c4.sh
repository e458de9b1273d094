#!/bin/bash
# The headline round and config 4's mean (the same k_reduce launches at 1000 x 25 M) in separate standalone
# processes, alternating, same steps: does the FedAvg reduce run at the same per-launch time in both?
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $ROOT; mkdir -p gpurun_out
for rep in 1 2 3; do
  for cfg in headline c4; do
    out=$(timeout -k 10 240 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-seconds 0 --no-other-configs 2>gpurun_out/ab_hc_err.log | grep '^{') || { echo "$cfg failed"; tail -5 gpurun_out/ab_hc_err.log; exit 1; }
    python -c "import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']; s=r.get('kernel_ms_split') or {}; print('$cfg', 'rep $rep', 'ms_per_step %.3f' % d['ms_per_step'], 'k_reduce_ms_per_launch %.4f' % (s.get('k_reduce', d['kernel_ms']) / r['launches_per_step'] if not s else s['k_reduce'] / s['k_reduce_launches']), 'frac %.4f' % r['frac'])" "$out"
  done
done
