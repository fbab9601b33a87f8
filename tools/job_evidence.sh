#!/bin/bash
# rocprofv3 kernel traces + FETCH/WRITE PMC for the non-headline BASELINE configurations
# (VERDICT r2 item 4), each followed by its per-kernel breakdown.
set -o pipefail
run() {  # tag kernel arch E M batch
    bash tools/profile_config.sh "$@" > gpurun_out/$1.log 2>&1 || { tail -5 gpurun_out/$1.log; return 1; }
    python tools/trace_breakdown.py $(ls gpurun_out/$1/trace/*kernel_trace.csv) --forwards 5:3 \
        --out gpurun_out/$1/breakdown.txt | sed -n 2,12p
}
run r50_e4m3 gemm_f8mx_kernel resnet50 4 3 512 && \
run r50_e3m4 gemm_tt16_kernel resnet50 3 4 512 && \
run r50_e2m5 gemm_tt_kernel resnet50 2 5 512 && \
run mb_e3m4 gemm_tt_kernel mobilenet_v2 3 4 512
