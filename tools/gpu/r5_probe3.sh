# round 5: (1) kernel trace of config 5 on one GPU, chain and chain-free (launch gaps and per-launch durations);
# (2) 100 s of back-to-back headline rounds with the card's telemetry (does the sustained rate decay?)
set -o pipefail
O=gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for ch in on off; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/r5_c5trace_$ch -o c5 --output-format csv -- python3 bench.py --config c5 --steps 2 --warmup 1 --sustain 0 --cpu-seconds 0 --no-other-configs --rest 0 --mean-chain $ch > $O/r5_c5trace_$ch.json 2> $O/r5_c5trace_$ch.err || { tail -20 $O/r5_c5trace_$ch.err; exit 1; }
done
echo traces ok
timeout -k 10 400 python3 bench.py --sustain 100 --no-other-configs --cpu-seconds 0 > $O/r5_sustain100.json 2> $O/r5_sustain100.err || { tail -20 $O/r5_sustain100.err; exit 1; }
echo sustain ok
