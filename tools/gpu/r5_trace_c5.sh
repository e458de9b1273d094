#!/bin/bash
# kernel trace (no counters) of config 5 at 100 M on one GPU, chain form and chain-free: per-launch durations and
# the gaps between launches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
for c in on off; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_c5_$c -o run -- python3 bench.py --config c5 --params 100000000 --steps 2 --warmup 1 --cpu-seconds 0 --sustain 0 --mean-chain $c --no-other-configs > $O/tr_c5_$c.log 2>&1 || { tail -20 $O/tr_c5_$c.log; exit 1; }
done
find $O/tr_c5_on $O/tr_c5_off -name "*kernel_trace.csv" | head
