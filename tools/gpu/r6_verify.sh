#!/bin/bash
# round 6, the tree the round ends with: GPU suite + smoke, then the default N = 1 line (roofline.traffic attached from
# the keyed PMC entry of this library)
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6v_pytest_gpu.log 2>&1 || { tail -40 $O/r6v_pytest_gpu.log; exit 1; }
tail -1 $O/r6v_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r6v_smoke.log 2>&1 || { tail -20 $O/r6v_smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py > $O/r6v_bench_n1.json 2> $O/r6v_bench_n1.err || { tail -30 $O/r6v_bench_n1.err; exit 1; }
echo bench ok
