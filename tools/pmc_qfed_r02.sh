#!/bin/bash
# Round-2 PMC passes over q-FedAvg phase 1 (bench.py --policy qfedavg, 1000 x 25M): VALU issue counters,
# then FETCH_SIZE and WRITE_SIZE in passes of their own (MI355X_MICROARCH.md's HBM recipe).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out
ARGS="--policy qfedavg --steps 3 --warmup 1 --cpu-seconds 0 --no-other-configs"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_qf_valu -o run -- python3 bench.py $ARGS > $OUT/pmc_qf_valu.log 2>&1 || { tail -5 $OUT/pmc_qf_valu.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_qf_fetch -o run -- python3 bench.py $ARGS > $OUT/pmc_qf_fetch.log 2>&1 || { tail -5 $OUT/pmc_qf_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_qf_write -o run -- python3 bench.py $ARGS > $OUT/pmc_qf_write.log 2>&1 || { tail -5 $OUT/pmc_qf_write.log; exit 1; }
find $OUT/pmc_qf_* -name "*counter_collection.csv"
