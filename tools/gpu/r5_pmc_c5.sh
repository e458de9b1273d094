# round 5: PMC traffic of config 5 on one GPU (10,000 x 100 M q-FedAvg, 22 passes), chain form and chain-free,
# FETCH_SIZE and WRITE_SIZE in separate passes
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ch in on off; do for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c -d $O/r5_pmc_c5_${ch}_$c -o pmc --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --sustain 0 --cpu-seconds 0 --no-other-configs --rest 0 --mean-chain $ch > $O/r5_pmc_c5_${ch}_$c.json 2> $O/r5_pmc_c5_${ch}_$c.err || { tail -20 $O/r5_pmc_c5_${ch}_$c.err; exit 1; }
  echo "$ch $c ok"
done; done
