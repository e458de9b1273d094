#!/bin/bash
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/alloc_reuse_probe.py > $O/r6_alloc_reuse_probe.log 2>&1 || { tail -20 $O/r6_alloc_reuse_probe.log; exit 1; }
cat $O/r6_alloc_reuse_probe.log
