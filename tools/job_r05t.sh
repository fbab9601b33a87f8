#!/bin/bash
# Round 5, step t: LDS-DMA-staged table-form depthwise (conv_tbsg_kernel, tbs = 2): tbx tests,
# MobileNetV2 E4M3 and config 3 (E5M2 v9) per form.
set -o pipefail
OUT=gpurun_out/r05t; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tbx.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for t in 1 2; do
    FP8A_TBS=$t timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-cpu-baseline > $OUT/mb_e4m3_tbs$t.json 2> $OUT/mb.err || exit 1
    FP8A_TBS=$t timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --batch 512 --no-cpu-baseline > $OUT/c3_v9_tbs$t.json 2> $OUT/c3.err || exit 1
    python -c "import json; a=json.load(open('$OUT/mb_e4m3_tbs$t.json')); b=json.load(open('$OUT/c3_v9_tbs$t.json')); print('tbs=$t', round(a['value'],1), round(b['value'],1))"
  done
done
