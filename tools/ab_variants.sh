#!/bin/bash
# A/B of kernel builds on the ResNet-18 layer set (run from the repo root on the GPU box).
#   bash tools/ab_variants.sh [--test] base v_x v_y ...   (v_x = fp8_quantization_amd/lib/v_x.so)
# --test first runs the E4M3 per-term / matrix-core tests against each variant.
set -o pipefail
L=$PWD/fp8_quantization_amd/lib
T=0; if [ "$1" = "--test" ]; then T=1; shift; fi
for v in "$@"; do
  if [ $v = base ]; then f=$L/libfp8approx.so; else f=$L/$v.so; fi
  if [ $T = 1 ]; then
    FP8A_LIB_PATH=$f timeout -k 10 300 python -m pytest tests/test_gpu_f8.py tests/test_gpu_f8mx.py -x -q \
      --timeout 120 --timeout-method thread > gpurun_out/ab_test_$v.txt 2>&1
    echo "$v tests rc=$? $(tail -1 gpurun_out/ab_test_$v.txt)"
  fi
  FP8A_LIB_PATH=$f timeout -k 10 120 python tools/gemm_bench.py --reps 5 > gpurun_out/ab_$v.txt 2>&1 || exit 1
  echo $v $(grep total gpurun_out/ab_$v.txt)
done
