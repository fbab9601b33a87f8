#!/bin/bash
# Round 5, step j: division-free quantizer step + pointwise (1x1) dense GEMM path: the whole GPU
# suite, then config 1 with the path on / off (FP8A_NO_PW1) and the 3-waves build (lib/dn_b3.so).
set -o pipefail
OUT=gpurun_out/r05j; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline \
      > $OUT/c1_$tag.json 2> $OUT/c1_$tag.err || { tail -5 $OUT/c1_$tag.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/c1_$tag.json')); print('c1 $tag', round(d['value'],1), round(d['ms_per_step'],3))"
}
for r in 1 2; do
  run pw1 FP8A_X=1 || exit 1
  run nopw1 FP8A_NO_PW1=1 || exit 1
  run pw1_b3 FP8A_LIB_PATH=fp8_quantization_amd/lib/dn_b3.so || exit 1
  run nopw1_b3 FP8A_LIB_PATH=fp8_quantization_amd/lib/dn_b3.so FP8A_NO_PW1=1 || exit 1
done
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/ > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
