#!/bin/bash
# tile-table kernel builds A/B (FP8A_LIB_PATH) on the ResNet-18 layer set: E2M5 (lut), E3M4
# no-comp with the f32 form forced (FP8A_NO_TT16=1), E3M4 comp (f16 form).
# Usage: bash tools/ab_tt.sh v_a v_b ...
set -o pipefail
L=$PWD/fp8_quantization_amd/lib
for v in "$@"; do
  f=$L/$v.so
  a=$(FP8A_LIB_PATH=$f timeout -k 10 120 python tools/gemm_bench.py --mode lut --reps 5 | grep total | cut -c1-40) || exit 1
  b=$(FP8A_NO_TT16=1 FP8A_LIB_PATH=$f timeout -k 10 120 python tools/gemm_bench.py --mode w2u --reps 5 | grep total | cut -c1-40) || exit 1
  c=$(FP8A_LIB_PATH=$f timeout -k 10 120 python tools/gemm_bench.py --mode w2s --reps 5 | grep total | cut -c1-40) || exit 1
  echo "$v E2M5 $a | E3M4-f32 $b | E3M4-comp $c"
done
