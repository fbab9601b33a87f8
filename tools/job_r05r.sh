#!/bin/bash
# Round 5, step r: emission constants from the image header (kernel arguments shrunk); the emitting
# gemm_f8mx_kernel instances at 5 vs 4 waves per SIMD (lib/emit4.so): chain tests, ResNet-18 A/B.
set -o pipefail
OUT=gpurun_out/r05r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_qin.py \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for lib in default emit4; do
    if [ $lib = default ]; then E="FP8A_X=1"; else E="FP8A_LIB_PATH=fp8_quantization_amd/lib/emit4.so"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/r18_$lib.json 2> $OUT/r18_$lib.err || { tail -3 $OUT/r18_$lib.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/r18_$lib.json')); r=d['roofline']; print('r18 $lib', round(d['value'],1), round(r['kernel_avg_ms'],4), round(r['kernel_frac'],4))"
  done
done
