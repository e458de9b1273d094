#!/bin/bash
# round 6: config 1's host round after the leaner arrival path (and as bench.py runs it, NUMA-bound)
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c1_profile_r6.py > $O/r6d_c1_profile.log 2>&1 || { tail -20 $O/r6d_c1_profile.log; exit 1; }
cat $O/r6d_c1_profile.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "zero_copy or c1 or parity or ingress or sharded or edges" > $O/r6d_pytest.log 2>&1 || { tail -30 $O/r6d_pytest.log; exit 1; }
tail -1 $O/r6d_pytest.log
