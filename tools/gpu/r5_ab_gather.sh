#!/bin/bash
# round 5: deferred q-FedAvg gathers folding the windows with one wave per client (new default) against the
# thread-per-client fold (QF_GATHER_WAVE=0): q-FedAvg tests on the new library (incl. the deferred-gather bit
# check), the c5 chain pair A/B, and a kernel trace of the new gather
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
bash tools/build_ab.sh base "-DQF_GATHER_WAVE=0" > $O/ab_build_base.log 2>&1 || { tail -5 $O/ab_build_base.log; exit 1; }
cp fedscale_amd/libfedagg.so fedscale_amd/ab/libfedagg_new.so
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_qfed_mean.py tests/test_gpu_properties.py tests/test_gpu_sharded.py -k "qfed or c5 or gather" > $O/r5_gather_tests.log 2>&1 || { tail -30 $O/r5_gather_tests.log; exit 1; }
echo "new: $(tail -1 $O/r5_gather_tests.log)"
for rep in 1 2; do for n in base new; do
  echo "== $n rep $rep"
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 300 python3 tools/chain_pair.py 100000000 12500000 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); nc=d['no_chain']
    print('P', d['params'], 'chain_region %.2f' % d['dominant_kernel_ms'], 'paired chain %.2f no_chain %.2f cost %.2f%% (%d each)' % (nc['chain_round_ms_paired'], nc['round_ms_paired'], nc['chain_cost_pct'], nc['rounds_each']))
" || exit 1
done; done 2>&1 | tee $O/r5_ab_gather.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_gw -o run -- python3 bench.py --config c5 --params 100000000 --steps 2 --warmup 1 --cpu-seconds 0 --sustain 0 --mean-chain on --no-other-configs > $O/tr_gw.log 2>&1 || { tail -20 $O/tr_gw.log; exit 1; }
python3 tools/trace_by_shape.py $(find $O/tr_gw -name "run_kernel_trace.csv" | head -1) 3 | grep gather > $O/r5_gather_trace.jsonl
cat $O/r5_gather_trace.jsonl | cut -c1-200
