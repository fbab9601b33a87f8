#!/bin/bash
# Round 5, step c: A/B of gemm_f8mx_kernel variants (FP8A_LIB_PATH) on the ResNet-18 layer set and
# the headline bench line; libraries named on the command line (lib/<name>.so).
set -o pipefail
OUT=gpurun_out/${OUTTAG:-r05c}; mkdir -p $OUT
L=fp8_quantization_amd/lib
for round in 1 2; do
  for v in "$@"; do
    FP8A_LIB_PATH=$L/$v.so timeout -k 10 300 python tools/gemm_bench.py --batch 256 --reps 5 > $OUT/layers_${v}_$round.log 2>&1 || exit $?
    echo "$v round $round $(tail -1 $OUT/layers_${v}_$round.log)"
  done
done
for v in "$@"; do
  FP8A_LIB_PATH=$L/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit $?
  echo "$v bench $(python -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(round(d['value'],1), round(d['roofline']['frac'],4))")"
done
