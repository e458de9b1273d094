#!/bin/bash
# the post-fill slowdown probe (tools/rest_probe.py), config 3 on one GPU
set -e
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/rest_probe.py > gpurun_out/r5_rest_probe.log 2>&1
