#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
STAGE=${1:-all}
run() { echo "== $*" ; }
if [[ $STAGE == all || $STAGE == test ]]; then
  run tests
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  run bench
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  run rocprof
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  tail -1 $OUT/prof.log
  find $OUT/prof -name "*kernel_stats.csv" | head -3
fi
