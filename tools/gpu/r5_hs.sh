#!/bin/bash
# round 5, library with the batched hs recurrence: GPU suite, smoke, a kernel trace of config 5's shard (k_qfed_hs at
# K = 10,000), PMC traffic of the headline for this build, and the headline under rocprofv3 --stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r5c_pytest_gpu.log 2>&1 || { tail -40 $O/r5c_pytest_gpu.log; exit 1; }
tail -1 $O/r5c_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5c_smoke.log 2>&1 || { tail -20 $O/r5c_smoke.log; exit 1; }
grep smoke $O/r5c_smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_hs -o run -- python3 bench.py --config c5 --params 12500000 --steps 3 --warmup 1 --cpu-seconds 0 --sustain 0 --no-other-configs > $O/tr_hs.log 2>&1 || { tail -20 $O/tr_hs.log; exit 1; }
python3 tools/trace_by_shape.py $(find $O/tr_hs -name "run_kernel_trace.csv" | head -1) 2 > $O/r5c_c5shard_trace.jsonl || exit 1
rm -f $(find $O/tr_hs -name "run_kernel_trace.csv")
grep "qfed_hs\|gather" $O/r5c_c5shard_trace.jsonl | cut -c1-200
H="bench.py --no-other-configs --cpu-seconds 0 --sustain 0"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d $O/r5c_pmc_head_$c -o pmc --output-format csv -- python3 $H --steps 3 --warmup 1 > $O/r5c_pmc_head_$c.json 2> $O/r5c_pmc_head_$c.err || { tail -20 $O/r5c_pmc_head_$c.err; exit 1; }
  echo "head $c ok"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5c_head_stats -o run -- python3 bench.py --no-other-configs --cpu-seconds 0 > $O/r5c_headline_under_rocprof.json 2> $O/r5c_head_stats.err || { tail -20 $O/r5c_head_stats.err; exit 1; }
rm -f $(find $O/r5c_head_stats -name "run_kernel_trace.csv")
echo stats ok
