#!/bin/bash
# is the one-GPU chain cost of config 5 a power-cap effect? (tools/chain_power_probe.py)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/chain_power_probe.py 100000000 4 > gpurun_out/r5_chain_power_100m.log 2>&1
timeout -k 10 200 python -u tools/chain_power_probe.py 12500000 4 > gpurun_out/r5_chain_power_shard.log 2>&1
