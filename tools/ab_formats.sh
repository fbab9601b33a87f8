#!/bin/bash
# A/B of the E3M4 / E2M5 path on the ResNet-18 layer set: gemm_tt_kernel vs gemm_fast_kernel
# (FP8A_NO_TT=1), every table mode (run from the repo root on the GPU box).
set -o pipefail
for m in w2u w2s lut w2s2; do
  timeout -k 10 180 python tools/gemm_bench.py --mode $m --reps 3 > gpurun_out/fmt_tt_$m.txt 2>&1 || exit 1
  FP8A_NO_TT=1 timeout -k 10 180 python tools/gemm_bench.py --mode $m --reps 3 > gpurun_out/fmt_old_$m.txt 2>&1 || exit 1
  echo "$m tt $(grep total gpurun_out/fmt_tt_$m.txt) old $(grep total gpurun_out/fmt_old_$m.txt)"
done
