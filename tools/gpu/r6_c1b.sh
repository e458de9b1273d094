#!/bin/bash
# round 6: config 1 after the arrival short path and the clones allocated before the wait; targeted GPU tests
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c1_profile_r6.py > $O/r6g_c1_profile.log 2>&1 || { tail -20 $O/r6g_c1_profile.log; exit 1; }
cat $O/r6g_c1_profile.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "zero_copy or c1 or parity or ingress or sharded or edges or smoke or adapter" > $O/r6g_pytest.log 2>&1 || { tail -30 $O/r6g_pytest.log; exit 1; }
tail -1 $O/r6g_pytest.log
