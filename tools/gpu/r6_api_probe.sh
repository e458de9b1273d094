#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/launch_api_probe.py > $O/r6_launch_api_probe.log 2>&1 || { tail -20 $O/r6_launch_api_probe.log; exit 1; }
cat $O/r6_launch_api_probe.log
