#!/bin/bash
# E3M4 tile-table kernel A/B: packed-f16 form (default) vs the f32 form (FP8A_NO_TT16=1), ResNet-18
# layer set, no-comp (w2u) and comp (w2s) tables.
set -o pipefail
for m in w2u w2s; do
  timeout -k 10 120 python tools/gemm_bench.py --mode $m --reps 5 > gpurun_out/tt16_$m.txt 2>&1 || exit 1
  FP8A_NO_TT16=1 timeout -k 10 120 python tools/gemm_bench.py --mode $m --reps 5 > gpurun_out/tt32_$m.txt 2>&1 || exit 1
  echo "$m f16: $(grep total gpurun_out/tt16_$m.txt | cut -c1-80)"
  echo "$m f32: $(grep total gpurun_out/tt32_$m.txt | cut -c1-80)"
done
