#!/bin/bash
# round 6, first probes: config 1's host round call by call (tools/c1_profile_r6.py); the q-FedAvg division power
# probe (tools/gpu/r6_div_power.sh); bench.py --gpus 2 and 8 as gloo ranks on the one card (plumbing: the N > 1
# line's fields, pcie_inclusive + cpu_baseline included)
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/c1_profile_r6.py > $O/r6_c1_profile.log 2>&1 || { tail -20 $O/r6_c1_profile.log; exit 1; }
cat $O/r6_c1_profile.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.2 --cpu-seconds 3 > $O/r6_rehearse_2.log 2>&1 || { tail -40 $O/r6_rehearse_2.log; exit 1; }
grep '^{' $O/r6_rehearse_2.log > $O/r6_bench_gloo_rehearsal_2.json
echo rehearsal2 ok
bash tools/gpu/r6_div_power.sh
