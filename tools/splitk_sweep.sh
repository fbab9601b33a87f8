#!/bin/bash
# per-layer time vs forced split-K factor
for S in 1 2 3 4 5 6 7 8; do
  FP8A_SPLITK=$S timeout -k 10 120 python tools/gemm_bench.py --reps 5 > gpurun_out/sk_$S.txt 2>&1 || exit 1
done
timeout -k 10 120 python tools/gemm_bench.py --reps 5 > gpurun_out/sk_auto.txt 2>&1
