# round 5: q-FedAvg column windows in one launch (QF_MULTIWIN / QF_CHAIN_MULTIWIN) against separate launches
set -o pipefail
O=gpurun_out; mkdir -p $O
( bash tools/build_ab.sh base "" > $O/ab_build_base.log 2>&1 ) &
( bash tools/build_ab.sh mw "-DQF_MULTIWIN=1 -DQF_CHAIN_MULTIWIN=1" > $O/ab_build_mw.log 2>&1 ) &
wait
ls fedscale_amd/ab/ || exit 1
FEDAGG_LIB=$PWD/fedscale_amd/ab/libfedagg_mw.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_edges.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_qfed_mean.py -k "qfed or c5" > $O/r5_mw_tests.log 2>&1 || { tail -30 $O/r5_mw_tests.log; exit 1; }
tail -1 $O/r5_mw_tests.log
bash tools/ab_c5.sh base mw 2>&1 | tee $O/r5_ab_mw_shard.log || exit 1
AB_PARAMS=100000000 AB_STEPS=2 AB_REPS=2 bash tools/ab_c5.sh base mw 2>&1 | tee $O/r5_ab_mw_100m.log || exit 1
AB_PARAMS=100000000 AB_STEPS=2 AB_REPS=1 AB_CHAIN=off bash tools/ab_c5.sh base mw 2>&1 | tee -a $O/r5_ab_mw_100m.log || exit 1
