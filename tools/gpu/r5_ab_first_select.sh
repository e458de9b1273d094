#!/bin/bash
# round 5: the chain-starting call's client 0 as an add onto -0 (new default) against round 4's per-element select
# (QF_FIRST_SELECT=1): q-FedAvg parity on the new library, then the chain cost at the power cap and paired, A/B.
set -o pipefail
O=gpurun_out; mkdir -p $O
bash tools/build_ab.sh sel "-DQF_FIRST_SELECT=1" > $O/ab_build_sel.log 2>&1 || { tail -5 $O/ab_build_sel.log; exit 1; }
cp fedscale_amd/libfedagg.so fedscale_amd/ab/libfedagg_new.so
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_qfed_mean.py -k "qfed or c5" > $O/r5_new_qfed_tests.log 2>&1 || { tail -30 $O/r5_new_qfed_tests.log; exit 1; }
echo "new: $(tail -1 $O/r5_new_qfed_tests.log)"
for rep in 1 2; do for n in sel new; do
  echo "== $n rep $rep"
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 200 python -u tools/chain_power_probe.py 100000000 4 2>/dev/null | tail -1 || exit 1
done; done 2>&1 | tee $O/r5_ab_first_select_cap.log
for rep in 1 2; do for n in sel new; do
  echo "== $n rep $rep"
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 300 python3 tools/chain_pair.py 100000000 12500000 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); nc=d['no_chain']
    print('P', d['params'], 'chain_region %.2f' % d['dominant_kernel_ms'], 'paired chain %.2f no_chain %.2f cost %.2f%%' % (nc['chain_round_ms_paired'], nc['round_ms_paired'], nc['chain_cost_pct']))
" || exit 1
done; done 2>&1 | tee $O/r5_ab_first_select_paired.log
