#!/bin/bash
# round 6: config 1's host round (wait modes, A/B of the small-round finish and of a polled egress wait) and the N = 1
# headline round through the drop-in against bench.Workload, interleaved
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c1_profile_r6.py > $O/r6c_c1_profile.log 2>&1 || { tail -20 $O/r6c_c1_profile.log; exit 1; }
cat $O/r6c_c1_profile.log
timeout -k 10 300 python -u tools/dropin_vs_workload.py > $O/r6c_dropin_vs_workload.log 2>&1 || { tail -20 $O/r6c_dropin_vs_workload.log; exit 1; }
cat $O/r6c_dropin_vs_workload.log
