#!/bin/bash
# Measurement pass on the GPU box (run from the repo root via gpurun):
#   bench (JSON line) -> rocprofv3 kernel trace + stats -> PMC passes (FETCH_SIZE, WRITE_SIZE,
#   SQ counters; each its own pass, kernel-trace only) -> tools/prof_summary.py.
# Usage: bash tools/gpu_profile.sh <round-tag> [steps]
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-5}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
LAUNCH_PER_STEP=21
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 > $OUT/bench.json 2> $OUT/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python $R/bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex gemm_f8mx -f csv -d $OUT/pmc_fetch -o run -- \
    python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex gemm_f8mx -f csv -d $OUT/pmc_write -o run -- \
    python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex gemm_f8mx -f csv -d $OUT/pmc_sq -o run -- \
    python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_sq.log 2>&1 ; \
cd $R && python tools/prof_summary.py --trace $(ls $OUT/trace/*kernel_trace.csv) --stats $(ls $OUT/trace/*kernel_stats.csv) \
    --pmc $(ls $OUT/pmc_*/*counter_collection.csv 2>/dev/null) --timed-launches $((STEPS*LAUNCH_PER_STEP)) \
    --out $OUT/summary --pmc-json $OUT/pmc.json --note "bench.py --steps $STEPS --warmup 2 (resnet18 E4M3 approx_v9, batch 512)" --batch 512 ; \
cat $OUT/bench.json
