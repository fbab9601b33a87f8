#!/bin/bash
# Round 5, step w: small exact convolutions on dn_direct_kernel (the stem): dense / fused-layer /
# MobileNetV2 tests, config 1 with dn_direct 1 / 0.
set -o pipefail
OUT=gpurun_out/r05w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dense.py \
    tests/test_gpu_grouped_conv.py tests/test_gpu_mbv2_layers.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for d in 1 0; do
    FP8A_DN_DIRECT=$d timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline \
        > $OUT/c1_direct$d.json 2> $OUT/c1.err || { tail -5 $OUT/c1.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/c1_direct$d.json')); print('c1 direct=$d', round(d['value'],1))"
  done
done
