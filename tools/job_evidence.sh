#!/bin/bash
# Bench lines for every BASELINE configuration + rocprofv3 evidence (trace + FETCH / WRITE) for the
# non-headline approx configurations.  Lines -> gpurun_out/ev/<name>.json.
set -o pipefail
OUT=gpurun_out/ev; mkdir -p $OUT
line() {  # name, bench args
    local n=$1; shift
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/$n.json 2> $OUT/$n.err || { tail -3 $OUT/$n.err; return 1; }
    python -c "import json; d=json.load(open('$OUT/$n.json')); r=d.get('roofline') or {}; print('$n', round(d['value'],1), r.get('frac'), r.get('traffic'))"
}
prof() {  # tag kernel arch E M batch [extra]
    bash tools/profile_config.sh "$@" > gpurun_out/$1.log 2>&1 || { tail -5 gpurun_out/$1.log; return 1; }
    python tools/trace_breakdown.py $(ls gpurun_out/$1/trace/*kernel_trace.csv) --forwards 5:3 \
        --out gpurun_out/$1/breakdown.txt | sed -n 2,8p
}
line c1_mbv2_noapprox --arch mobilenet_v2 --no-approx --batch 256 && \
line c3_mbv2_e5m2_v5 --arch mobilenet_v2 --expo-width 5 --mant-width 2 --v5-ofuf && \
line c4_vit_b16 --arch vit_b16 && \
line c5_r50_e4m3 --arch resnet50 && \
line c5_r50_e3m4 --arch resnet50 --expo-width 3 --mant-width 4 && \
line c5_r50_e2m5 --arch resnet50 --expo-width 2 --mant-width 5 && \
line c5_r50_e5m2 --arch resnet50 --expo-width 5 --mant-width 2 && \
prof r50_e4m3_r3 gemm_f8mx_kernel resnet50 4 3 512 && \
prof r50_e3m4_r3 gemm_tt16_kernel resnet50 3 4 512 && \
prof r50_e2m5_r3 gemm_tt_kernel resnet50 2 5 512 && \
prof mb_e3m4_r3 gemm_tt_kernel mobilenet_v2 3 4 512
