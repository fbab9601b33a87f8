#!/bin/bash
# per-layer time vs forced split-K factor: bash tools/splitk_sweep.sh [batch]
B=${1:-256}
for S in 1 2 3 4 5 6 7 8; do
  FP8A_SPLITK=$S timeout -k 10 120 python tools/gemm_bench.py --batch $B --reps 5 > gpurun_out/sk_${B}_$S.txt 2>&1 || exit 1
done
timeout -k 10 120 python tools/gemm_bench.py --batch $B --reps 5 > gpurun_out/sk_${B}_auto.txt 2>&1
