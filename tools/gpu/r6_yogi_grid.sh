#!/bin/bash
# round 6: k_yogi_step grid cap and per-thread unroll (FA_YOGI_GRID_MAX / FA_YOGI_U: knobs added for this sweep, removed
# after it; tuning builds from
# tools/build_ab.sh), each library in its own process, three interleaved passes, at config 4's per-GPU sizes
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
: > $O/r6_yogi_grid.log
for pass in 1 2 3; do
  for lib in fedscale_amd/ab/libfedagg_yg*.so; do
    FEDAGG_LIB=$lib timeout -k 10 90 python -u tools/yogi_step_probe.py 25000000 6250048 3125056 >> $O/r6_yogi_grid.log 2>> $O/r6_yogi_grid.err || { tail -20 $O/r6_yogi_grid.err; exit 1; }
  done
done
