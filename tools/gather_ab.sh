#!/bin/bash
# A/B of the host gather's streaming stores (FEDAGG_GATHER_NT), interleaved runs of tools/gather_probe.py
set -o pipefail
for i in 1 2 3; do
  for nt in 1 0; do
    FEDAGG_GATHER_NT=$nt timeout -k 10 120 python tools/gather_probe.py ${WORKERS:-1,4,8,16,24} 2>/dev/null | grep '^{' || exit 1
  done
done
