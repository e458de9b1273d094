#!/bin/bash
# VERDICT r5 #3 (one time-boxed attempt): is the q-FedAvg division's energy what clocks config 5's one-GPU chain
# rounds down at the 1400 W cap?  The product library and a tuning build whose fast_div is a bare multiply by RN(1/lr)
# (QF_DIV_MUL=1, wrong bits: power / clock / time only), each through tools/chain_power_probe.py (chain and chain-free
# regions alternating over the same resident uploads, the card's power and shader clock per region).
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 bash tools/build_ab.sh divmul "-DFA_TUNING=1 -DQF_DIV_MUL=1" > $O/r6_div_build.log 2>&1 || { tail -20 $O/r6_div_build.log; exit 1; }
timeout -k 10 300 python -u tools/chain_power_probe.py 100000000 4 > $O/r6_div_power_product.log 2>&1 || { tail -20 $O/r6_div_power_product.log; exit 1; }
FEDAGG_LIB=$GRAFT_REPO_ROOT/fedscale_amd/ab/libfedagg_divmul.so timeout -k 10 300 python -u tools/chain_power_probe.py 100000000 4 > $O/r6_div_power_mul.log 2>&1 || { tail -20 $O/r6_div_power_mul.log; exit 1; }
timeout -k 10 300 python -u tools/chain_power_probe.py 100000000 4 > $O/r6_div_power_product2.log 2>&1 || { tail -20 $O/r6_div_power_product2.log; exit 1; }
tail -1 $O/r6_div_power_product.log $O/r6_div_power_mul.log $O/r6_div_power_product2.log
