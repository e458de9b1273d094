set -o pipefail
B="python bench.py --no-other-configs --cpu-seconds 0 --steps 5 --warmup 1"
for spec in "qfedavg 1000 25000000" "qfedavg 462 25000000" "qfedavg 462 50000000" "qfedavg 462 100000000" "qfedavg 231 100000000" "fedavg 462 100000000"; do
  set -- $spec
  timeout -k 10 200 $B --policy $1 --clients $2 --params $3 > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/probe.log') if l.startswith('{')][-1]); print('$spec', round(d['ms_per_step'],3), 'ms', round(d['hbm_gbps']), 'GB/s kernel')"
done
