# round 5: the q-FedAvg chain held in LDS (QF_CHAIN_CLDS, register-load tiles of 16 / 12 float4) against the 8-wide
# LDS-DMA chain tiles: bit checks, then config 5's chain cost paired per library (tools/chain_pair.py)
set -o pipefail
O=gpurun_out; mkdir -p $O
for v in "base:" "cl16:-DQF_CHAIN_CLDS=1 -DQF_CHAIN_V=16 -DQF_CHAIN_GLDS=0" "cl12:-DQF_CHAIN_CLDS=1 -DQF_CHAIN_V=12 -DQF_CHAIN_GLDS=0"; do
  n=${v%%:*}; d=${v#*:}
  ( bash tools/build_ab.sh $n "$d" > $O/ab_build_$n.log 2>&1 ) &
done
wait
ls fedscale_amd/ab || exit 1
for n in cl16 cl12; do
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_qfed_mean.py -k "qfed or c5" > $O/r5_${n}_tests.log 2>&1 || { tail -30 $O/r5_${n}_tests.log; exit 1; }
  echo "$n: $(tail -1 $O/r5_${n}_tests.log)"
done
for rep in 1 2; do for n in base cl16 cl12; do
  echo "== $n rep $rep"
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 300 python3 tools/chain_pair.py 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); nc=d['no_chain']
    print('P', d['params'], 'chain_region %.2f' % d['dominant_kernel_ms'], 'paired chain %.2f no_chain %.2f cost %.2f%%' % (nc['chain_round_ms_paired'], nc['round_ms_paired'], nc['chain_cost_pct']))
" || exit 1
done; done 2>&1 | tee $O/r5_ab_clds.log
