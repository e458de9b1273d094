#!/bin/bash
# the default line with the auto warmup (>= 1 s of rounds before the headline's timed region), then the same
# command with --warmup 3 (the old default) for comparison on the same box
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 420 python -u bench.py > $O/r5x_bench_n1.json 2> $O/r5x_bench_n1.err || { tail -30 $O/r5x_bench_n1.err; exit 1; }
timeout -k 10 200 python -u bench.py --warmup 3 --no-other-configs --cpu-seconds 0 > $O/r5x_bench_n1_w3.json 2> $O/r5x_bench_n1_w3.err || { tail -30 $O/r5x_bench_n1_w3.err; exit 1; }
echo bench ok
