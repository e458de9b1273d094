#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c1_profile_r6.py > $O/r6s_c1_profile.log 2>&1 || { tail -20 $O/r6s_c1_profile.log; exit 1; }
head -3 $O/r6s_c1_profile.log
