#!/bin/bash
# Round 5, step e: config-1 fused-layer / fused-qin / depthwise tests, the depthwise staging A/B
# (FP8A_DW3 = 1 register-staged, 2 LDS-DMA) on config 1, and evidence for configs 3 (v5) / 5 (E3M4).
set -o pipefail
OUT=gpurun_out/r05e; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grouped_conv.py \
    tests/test_gpu_mbv2_layers.py tests/test_gpu_qin.py tests/test_gpu_v5.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for dw in 1 2 1 2; do
  FP8A_DW3=$dw timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline \
      > $OUT/c1_dw$dw.json 2> $OUT/c1_dw$dw.err || { tail -5 $OUT/c1_dw$dw.err; exit 1; }
  echo "dw3=$dw $(cut -c1-110 $OUT/c1_dw$dw.json)"
done
bash tools/job_evidence_r05.sh c3_mbv2_e5m2_v5 c5_r50_e3m4
