#!/bin/bash
# round 6: the GPU suite after the config-1 host-path changes (native staging, small-round finish, join on the commit
# event), config 1 call by call again, and the default N = 1 line
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r6b_pytest_gpu.log 2>&1 || { tail -40 $O/r6b_pytest_gpu.log; exit 1; }
tail -1 $O/r6b_pytest_gpu.log
timeout -k 10 200 python -u tools/c1_profile_r6.py > $O/r6b_c1_profile.log 2>&1 || { tail -20 $O/r6b_c1_profile.log; exit 1; }
cat $O/r6b_c1_profile.log
timeout -k 10 600 python -u bench.py > $O/r6b_bench_n1.json 2> $O/r6b_bench_n1.err || { tail -30 $O/r6b_bench_n1.err; exit 1; }
python - <<'PY'
import json
l = json.loads(open("gpurun_out/r6b_bench_n1.json").read().splitlines()[-1])
o = l["other_configs"]
print("value", round(l["value"]), "frac", round(l["roofline"]["frac"], 4), "schema", l["schema"])
print("c1", o["c1_femnist_cnn_k10_host_round"]["round_ms_incl_h2d_d2h"], o["c1_femnist_cnn_k10_host_round"]["cpu_baseline"]["handler_round_ms"])
print("c5 chain", o["c5_qfedavg_k10000_p100M"]["round_ms"], o["c5_qfedavg_k10000_p100M"].get("no_chain", {}).get("chain_cost_pct"))
print("drop_in", l.get("value_drop_in"), "pcie", l["pcie_inclusive"]["host_to_device_GBps"])
PY
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 5 --warmup 2 --dist-backend gloo --mem-fraction 0.06 --cpu-seconds 3 > $O/r6b_rehearse_8.log 2>&1 || { tail -40 $O/r6b_rehearse_8.log; exit 1; }
grep '^{' $O/r6b_rehearse_8.log > $O/r6_bench_gloo_rehearsal_8.json
echo rehearsal8 ok
