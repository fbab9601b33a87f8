#!/bin/bash
# rocprofv3 evidence for one bench configuration (run from the repo root via gpurun):
#   kernel trace + stats of the bench run, then FETCH_SIZE, WRITE_SIZE and SQ (wave-cycle / VALU)
#   passes (each its own run, kernel-trace only) over the dominant kernel -> tools/prof_summary.py ->
#   gpurun_out/<tag>/{summary.json,summary.txt,pmc.json}.
# Usage: bash tools/profile_config.sh <tag> <kernel> <arch> <E> <M> <batch> [extra bench args]
set -o pipefail
TAG=$1; KERNEL=$2; ARCH=$3; E=$4; M=$5; BATCH=$6; shift 6
EXTRA="$*"
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
BENCH="$R/bench.py --arch $ARCH --expo-width $E --mant-width $M --batch $BATCH --no-cpu-baseline $EXTRA"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python $BENCH --steps 3 --warmup 1 > $OUT/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex $KERNEL -f csv -d $OUT/pmc_fetch -o run -- \
    python $BENCH --steps 2 --warmup 1 > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex $KERNEL -f csv -d $OUT/pmc_write -o run -- \
    python $BENCH --steps 2 --warmup 1 > $OUT/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex $KERNEL -f csv \
    -d $OUT/pmc_sq -o run -- python $BENCH --steps 2 --warmup 1 > $OUT/pmc_sq.log 2>&1 && \
cd $R && python tools/prof_summary.py --trace $(ls $OUT/trace/*kernel_trace.csv) --stats $(ls $OUT/trace/*kernel_stats.csv) \
    --pmc $(ls $OUT/pmc_*/*counter_collection.csv) --forwards 5:3,4:2 --kernel $KERNEL \
    --out $OUT/summary --pmc-json $OUT/pmc.json --arch $ARCH --E $E --M $M --batch $BATCH \
    --note "bench.py --arch $ARCH E${E}M${M} --batch $BATCH $EXTRA (trace: --steps 3 --warmup 1 + calibration; PMC: --steps 2 --warmup 1)"
