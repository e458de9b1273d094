# round 5, last tree: smoke() and the default line (no rest between regions; per-config card telemetry)
set -o pipefail
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r5g_smoke.log 2>&1 || { tail -20 $O/r5g_smoke.log; exit 1; }
grep smoke $O/r5g_smoke.log
timeout -k 10 420 python -u bench.py > $O/r5g_bench_n1.json 2> $O/r5g_bench_n1.err || { tail -30 $O/r5g_bench_n1.err; exit 1; }
echo bench ok
