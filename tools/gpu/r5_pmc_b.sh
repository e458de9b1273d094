#!/bin/bash
# round 5, library 59fb... (the wave-per-client window gather): PMC traffic of the headline and of config 5 on one
# GPU (chain form and chain-free), FETCH_SIZE and WRITE_SIZE in separate passes, then the headline under
# rocprofv3 --kernel-trace --stats
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
H="bench.py --no-other-configs --cpu-seconds 0 --sustain 0"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d $O/r5b_pmc_head_$c -o pmc --output-format csv -- python3 $H --steps 3 --warmup 1 > $O/r5b_pmc_head_$c.json 2> $O/r5b_pmc_head_$c.err || { tail -20 $O/r5b_pmc_head_$c.err; exit 1; }
  echo "head $c ok"
done
for ch in on off; do for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d $O/r5b_pmc_c5_${ch}_$c -o pmc --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --sustain 0 --cpu-seconds 0 --no-other-configs --rest 0 --mean-chain $ch > $O/r5b_pmc_c5_${ch}_$c.json 2> $O/r5b_pmc_c5_${ch}_$c.err || { tail -20 $O/r5b_pmc_c5_${ch}_$c.err; exit 1; }
  echo "c5 $ch $c ok"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r5b_head_stats -o run -- python3 bench.py --no-other-configs --cpu-seconds 0 > $O/r5b_headline_under_rocprof.json 2> $O/r5b_head_stats.err || { tail -20 $O/r5b_head_stats.err; exit 1; }
rm -f $(find $O/r5b_head_stats -name "run_kernel_trace.csv")
echo stats ok
