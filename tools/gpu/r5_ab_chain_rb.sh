#!/bin/bash
# round 5: chain launches with a register double buffer (QF_CHAIN_GLDS=-1: the next client loads while this one computes) against the LDS-DMA default
set -o pipefail
O=gpurun_out; mkdir -p $O
for v in "base:" "rb:-DQF_CHAIN_GLDS=-1"; do
  n=${v%%:*}; d=${v#*:}
  ( bash tools/build_ab.sh $n "$d" > $O/ab_build_$n.log 2>&1 ) &
done
wait
ls fedscale_amd/ab/libfedagg_base.so fedscale_amd/ab/libfedagg_rb.so || exit 1
FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_rb.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_qfed_mean.py -k "qfed or c5" > $O/r5_rb_tests.log 2>&1 || { tail -30 $O/r5_rb_tests.log; exit 1; }
echo "rb: $(tail -1 $O/r5_rb_tests.log)"
for rep in 1 2; do for n in base rb; do
  echo "== $n rep $rep"
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 300 python3 tools/chain_pair.py 100000000 12500000 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); nc=d['no_chain']
    print('P', d['params'], 'chain_region %.2f' % d['dominant_kernel_ms'], 'paired chain %.2f no_chain %.2f cost %.2f%% (%d each)' % (nc['chain_round_ms_paired'], nc['round_ms_paired'], nc['chain_cost_pct'], nc['rounds_each']))
" || exit 1
done; done 2>&1 | tee $O/r5_ab_chain_rb.log
