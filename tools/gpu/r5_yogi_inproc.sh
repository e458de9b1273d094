# round 5: k_yogi_step variants (nt loads/stores, float4 per thread), and the in-process round's host cost
# (8 parts on one card, tiny K, so the GPU time per round is small and the host's share shows)
set -o pipefail
O=gpurun_out; mkdir -p $O
for v in "base:" "nt:-DFA_YOGI_NT=1" "v2:-DFA_YOGI_V=2" "v2nt:-DFA_YOGI_V=2 -DFA_YOGI_NT=1"; do
  n=${v%%:*}; d=${v#*:}
  ( bash tools/build_ab.sh $n "$d" > $O/ab_build_$n.log 2>&1 ) &
done
wait
ls fedscale_amd/ab || exit 1
for rep in 1 2; do for n in base nt v2 v2nt; do
  FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_$n.so timeout -k 10 120 python3 tools/yogi_step_probe.py | tee -a $O/r5_yogi_step_probe.log || exit 1
done; done
for K in 20 200; do
  timeout -k 10 300 python3 -m fedscale_amd.inproc_bench --devices 0,0,0,0,0,0,0,0 --clients $K --params 25000000 --rounds 50 --warmup 5 --no-one-gpu | tee -a $O/r5_inproc_host_cost.log || exit 1
done
timeout -k 10 300 python3 -m fedscale_amd.inproc_bench --devices 0 --clients 20 --params 25000000 --rounds 50 --warmup 5 --no-one-gpu | tee -a $O/r5_inproc_host_cost.log || exit 1
