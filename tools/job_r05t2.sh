#!/bin/bash
# Round 5: kernel trace of the ViT-B/16 line (eager) with the GELU tail fused into the MLP's first
# linear, to price the fused epilogue against the separate GELU + quantize passes it replaces.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r05t2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python $R/bench.py --arch vit_b16 --batch 64 --no-cpu-baseline --no-graph --steps 3 --warmup 1 > $OUT/trace.log 2>&1 || exit 1
cd $R && python tools/trace_breakdown.py $(ls $OUT/trace/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown.txt > /dev/null && sed -n 1,22p $OUT/breakdown.txt
