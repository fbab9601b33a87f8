#!/bin/bash
# Round 5, step v: v5 depthwise -> projection word-image hand-off: chain / v5 / qin tests, config 3 v5
# with the chain on and off.
set -o pipefail
OUT=gpurun_out/r05v; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_v5.py \
    tests/test_gpu_qin.py tests/test_gpu_mbv2_layers.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for c in 1 0; do
    FP8A_CHAIN=$c timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --batch 512 --v5-ofuf \
        --no-cpu-baseline > $OUT/c3_chain$c.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c3_chain$c.json')); print('c3 v5 chain=$c', round(d['value'],1))"
  done
done
