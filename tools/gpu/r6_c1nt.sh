#!/bin/bash
# round 6: config 1 with streaming (non-temporal) staging copies against plain ones (A/B), call by call
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c1_profile_r6.py > $O/r6e_c1_profile.log 2>&1 || { tail -20 $O/r6e_c1_profile.log; exit 1; }
cat $O/r6e_c1_profile.log
