# round 5: small q-FedAvg chain calls (K <= QF_CHAIN_SMALLK) on a kernel with LDS for 4 x 1024 norms, so two
# workgroups fit per CU (grid 512, 4 M-column windows), against the default: bit checks, then the paired chain cost
set -o pipefail
O=gpurun_out; mkdir -p $O
for v in "base:" "w8:-DQF_CHAIN_W8=1"; do
  n=${v%%:*}; d=${v#*:}
  ( bash tools/build_ab.sh $n "$d" > $O/ab_build_$n.log 2>&1 ) &
done
wait
ls fedscale_amd/ab || exit 1
for n in w8; do
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_qfed_mean.py -k "qfed or c5" > $O/r5_${n}_tests.log 2>&1 || { tail -30 $O/r5_${n}_tests.log; exit 1; }
  echo "$n: $(tail -1 $O/r5_${n}_tests.log)"
done
for rep in 1 2 3; do for n in base w8; do
  echo "== $n rep $rep"
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 300 python3 tools/chain_pair.py 100000000 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); nc=d['no_chain']
    if d['params'] < 50_000_000: continue
    print('P', d['params'], 'chain_region %.2f' % d['dominant_kernel_ms'], 'paired chain %.2f no_chain %.2f cost %.2f%%' % (nc['chain_round_ms_paired'], nc['round_ms_paired'], nc['chain_cost_pct']))
" || exit 1
done; done 2>&1 | tee $O/r5_ab_chain_w8.log
