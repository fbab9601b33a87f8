#!/bin/bash
# Round 5 (af): af32_maxct (1x1 convs / matrices with at most this many column tiles stage A as
# fp32 inside gemm_f8mx_kernel instead of the A pre-pass) re-measured now that the pre-pass keeps
# 4 loads in flight: MobileNetV2 E4M3 / E5M2 v9 and ResNet-50 E4M3, eager lines.
set -o pipefail
OUT=gpurun_out/r05af; mkdir -p $OUT
for cfg in "e4m3 mobilenet_v2 4 3 512" "v9 mobilenet_v2 5 2 512" "r50 resnet50 4 3 512"; do
  set -- $cfg; T=$1; shift
  for mc in 3 0 1 3 0; do
    FP8A_AF32_MAXCT=$mc timeout -k 10 300 python bench.py --arch $1 --expo-width $2 --mant-width $3 --batch $4 --no-cpu-baseline \
        --no-graph > $OUT/${T}_mc$mc.json 2> $OUT/${T}_mc$mc.err || { tail -3 $OUT/${T}_mc$mc.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${T}_mc$mc.json')); print('$T maxct $mc', round(d['value'],1))"
  done
done
