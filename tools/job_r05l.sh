#!/bin/bash
# Round 5, step l: fq_apply_fast in the dense GEMM's A loads / epilogue and the depthwise store.
set -o pipefail
OUT=gpurun_out/r05l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dense.py \
    tests/test_gpu_grouped_conv.py tests/test_gpu_mbv2_layers.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline > $OUT/c1_$r.json 2> $OUT/c1_$r.err || exit 1
  python -c "import json; d=json.load(open('$OUT/c1_$r.json')); r=d['roofline']; print('c1', round(d['value'],1), r.get('kernel_avg_ms'))"
done
