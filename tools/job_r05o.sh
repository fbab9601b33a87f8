#!/bin/bash
# Round 5, step o: staged v5 depthwise (conv_v5ds_kernel): v5 / qin / MobileNetV2-layer tests, config 3 v5.
set -o pipefail
OUT=gpurun_out/r05o; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_v5.py \
    tests/test_gpu_qin.py tests/test_gpu_mbv2_layers.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in 1 0; do
  FP8A_V5DS=$v timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --batch 512 --v5-ofuf \
      --no-cpu-baseline > $OUT/c3_v5ds$v.json 2> $OUT/c3_v5ds$v.err || { tail -5 $OUT/c3_v5ds$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c3_v5ds$v.json')); print('c3 v5ds=$v', round(d['value'],1))"
done
