#!/bin/bash
# round 6: the whole default bench run under rocprofv3 (kernel trace + stats): every config's kernels, final library
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/r6_prof_all -o all --output-format csv -- python3 bench.py > $O/r6_prof_all_bench.json 2> $O/r6_prof_all.err || { tail -20 $O/r6_prof_all.err; exit 1; }
head -20 $O/r6_prof_all/all_kernel_stats.csv
gzip -c $O/r6_prof_all/all_kernel_trace.csv > $O/r6_prof_all_kernel_trace.csv.gz
