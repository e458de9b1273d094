#!/bin/bash
# round 6: the round-end GPU tier on the current tree — pytest -m gpu (one process), then smoke()
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rs > $O/r6_pytest_gpu.log 2>&1 || { tail -40 $O/r6_pytest_gpu.log; exit 1; }
tail -3 $O/r6_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r6_smoke.log 2>&1 || { tail -20 $O/r6_smoke.log; exit 1; }
grep smoke $O/r6_smoke.log
