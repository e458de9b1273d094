#!/bin/bash
# round 6, last pass on the final tree: the GPU suite + smoke, config 1 call by call, the default N = 1 line
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6m_pytest_gpu.log 2>&1 || { tail -40 $O/r6m_pytest_gpu.log; exit 1; }
tail -1 $O/r6m_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r6m_smoke.log 2>&1 || { tail -20 $O/r6m_smoke.log; exit 1; }
timeout -k 10 300 python -u tools/c1_profile_r6.py > $O/r6m_c1_profile.log 2>&1 || { tail -20 $O/r6m_c1_profile.log; exit 1; }
head -3 $O/r6m_c1_profile.log
timeout -k 10 600 python -u bench.py > $O/r6m_bench_n1.json 2> $O/r6m_bench_n1.err || { tail -30 $O/r6m_bench_n1.err; exit 1; }
echo bench ok
