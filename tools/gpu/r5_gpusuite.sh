#!/bin/bash
# the round-end GPU tier on the current tree: pytest -m gpu (one process), then smoke()
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r5_pytest_gpu.log 2>&1 || { tail -40 $O/r5_pytest_gpu.log; exit 1; }
tail -1 $O/r5_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5_smoke.log 2>&1 || { tail -20 $O/r5_smoke.log; exit 1; }
grep smoke $O/r5_smoke.log
