#!/bin/bash
# rocprofv3 kernel trace + stats of the whole default bench.py run (every config), summarised per (kernel, grid)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_all -o run -- python3 bench.py > $O/r5_prof_all_bench.json 2> $O/r5_prof_all_bench.err || { tail -30 $O/r5_prof_all_bench.err; exit 1; }
T=$(find $O/prof_all -name "run_kernel_trace.csv" | head -1)
python3 tools/trace_by_shape.py $T 3 > $O/r5_prof_all_by_shape.jsonl || exit 1
cp $(find $O/prof_all -name "run_kernel_stats.csv" | head -1) $O/r5_prof_all_kernel_stats.csv || exit 1
gzip -c $T > $O/r5_prof_all_kernel_trace.csv.gz && rm -f $T
head -30 $O/r5_prof_all_by_shape.jsonl | cut -c1-220
