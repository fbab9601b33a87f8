#!/bin/bash
# Round 5, step d: the persistent depthwise kernels -- bit-identity tests, configs 1 / MobileNetV2
# E4M3 / config 3 v9 bench lines; the E3M4 layer set (round-3 reference: 56.4 ms no-comp).
set -o pipefail
OUT=gpurun_out/${1:-r05d}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_grouped_conv.py tests/test_gpu_tbx.py tests/test_gpu_mbv2_layers.py -q -x \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
for spec in "c1:--arch mobilenet_v2 --no-approx" "mb_e4m3:--arch mobilenet_v2" "c3_v9:--arch mobilenet_v2 --expo-width 5 --mant-width 2"; do
  tag=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline --steps 10 > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit $?
  echo "$tag $(python -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print(round(d['value'],1))")"
done
timeout -k 10 300 python tools/gemm_bench.py --mode w2u --reps 3 > $OUT/layers_e3m4.log 2>&1 || exit $?
tail -1 $OUT/layers_e3m4.log
