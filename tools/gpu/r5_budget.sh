#!/bin/bash
# config 5 on one GPU with 0.6 (bench default) and 0.8 of the free HBM for the resident uploads: passes, round time,
# chain cost (paired as bench.py does, then at the power cap back to back)
set -o pipefail
O=gpurun_out; mkdir -p $O
for rep in 1 2; do for b in 0.6 0.8; do
  echo "== budget $b rep $rep"
  timeout -k 10 300 python3 tools/chain_pair.py 100000000 budget=$b 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); nc=d['no_chain']
    print('P', d['params'], 'C', d['resident_clients'], 'passes', d['passes'], 'round %.2f' % d['round_ms'], 'paired chain %.2f no_chain %.2f cost %.2f%%' % (nc['chain_round_ms_paired'], nc['round_ms_paired'], nc['chain_cost_pct']))
" || exit 1
done; done 2>&1 | tee $O/r5_budget_paired.log
for b in 0.6 0.8; do
  echo "== cap, budget $b"
  timeout -k 10 200 python -u tools/chain_power_probe.py 100000000 4 $b 2>/dev/null | grep -v '"region"' || exit 1
done 2>&1 | tee $O/r5_budget_cap.log
