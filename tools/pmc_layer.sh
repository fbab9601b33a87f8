#!/bin/bash
# PMC counters of the fast kernel on one ResNet-18 layer (tools/gemm_bench.py), separate passes.
# Usage: bash tools/pmc_layer.sh <tag> <mode> <layer>
TAG=$1; MODE=${2:-w1u}; LAYER=${3:-l2.c2}
R=$(pwd); OUT=$R/gpurun_out/pmc_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { timeout -k 10 300 rocprofv3 --kernel-trace --pmc $2 --kernel-include-regex ${KREGEX:-gemm_f8mx} -f csv -d $OUT/$1 -o run -- \
        python $R/tools/gemm_bench.py --mode $MODE --layers $LAYER --reps 3 > $OUT/$1.log 2>&1; }
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" && \
run sq2 "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM" && \
run grbm "GRBM_GUI_ACTIVE GRBM_COUNT"
cd $R && python - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]; acc = collections.defaultdict(list)
for f in glob.glob(out + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc): print(f"{k:28s} {sum(acc[k]) / len(acc[k]):.4g}")
PY
