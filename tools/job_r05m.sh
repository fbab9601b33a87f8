#!/bin/bash
# Round 5, step m: quantizer form A/B (fq_apply_fast vs the literal form: lib/fqlit.so) on the
# fake-quant kernel, the depthwise layer set and config 1.
set -o pipefail
OUT=gpurun_out/r05m; mkdir -p $OUT
for lib in default fqlit; do
  if [ $lib = default ]; then E=""; else E="FP8A_LIB_PATH=fp8_quantization_amd/lib/fqlit.so"; fi
  env $E timeout -k 10 120 python tools/fq_bench.py > $OUT/fq_$lib.log 2>&1 || { tail -3 $OUT/fq_$lib.log; exit 1; }
  echo "fq $lib $(tail -1 $OUT/fq_$lib.log)"
  env $E timeout -k 10 300 python tools/dw_bench.py --dw3 2 --qin > $OUT/dw_$lib.log 2>&1 || exit 1
  echo "dw $lib $(tail -1 $OUT/dw_$lib.log | cut -c1-60)"
  env $E timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline > $OUT/c1_$lib.json 2> $OUT/c1_$lib.err || exit 1
  python -c "import json; d=json.load(open('$OUT/c1_$lib.json')); r=d['roofline']; print('c1 $lib', round(d['value'],1), r.get('kernel_avg_ms'))"
done
