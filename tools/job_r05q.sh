#!/bin/bash
# Round 5, step q: tile-table kernels without the word-image emission code (store_tile<false>):
# tt tests, E3M4 / E2M5 layer sets, ResNet-50 E3M4 / E2M5 evidence.
set -o pipefail
OUT=gpurun_out/r05q; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tt.py tests/test_gpu_chain.py \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for m in w2u lut; do
  timeout -k 10 300 python tools/gemm_bench.py --mode $m --reps 5 > $OUT/$m.log 2>&1 || exit 1
  echo "$m $(tail -1 $OUT/$m.log)"
done
bash tools/job_evidence_r05.sh c5_r50_e3m4 c5_r50_e2m5
