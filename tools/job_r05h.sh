#!/bin/bash
# Round 5, step h: bit-level fq_apply + quad depthwise (dn_dw3g_kernel): quantizer / depthwise / qin
# tests, the depthwise layer set per form, config-1 bench per form.
set -o pipefail
OUT=gpurun_out/r05h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_grouped_conv.py tests/test_gpu_qin.py tests/test_gpu_mbv2_layers.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for dw in 1 2; do
  timeout -k 10 300 python tools/dw_bench.py --dw3 $dw --qin > $OUT/dw_$dw.log 2>&1 || { tail -5 $OUT/dw_$dw.log; exit 1; }
  echo "dw3=$dw $(tail -1 $OUT/dw_$dw.log)"
done
for dw in 1 2 1 2; do
  FP8A_DW3=$dw timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline \
      > $OUT/c1_dw$dw.json 2> $OUT/c1_dw$dw.err || { tail -5 $OUT/c1_dw$dw.err; exit 1; }
  echo "c1 dw3=$dw $(cut -c1-130 $OUT/c1_dw$dw.json | cut -d, -f2)"
done
