#!/bin/bash
# Round 5 (z): the two-slot flag arena (the last kernel of a launch zeroes the other slot): arena
# and fallback tests, then eager A/B lines against the pre-arena library (_ab/lib_before.so) on
# E5M2 v9, E4M3 MobileNetV2, v5 and ViT.
set -o pipefail
OUT=gpurun_out/r05z; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f8mx.py tests/test_gpu_tbx.py \
    tests/test_gpu_f8_e5m2.py tests/test_gpu_v5.py tests/test_gpu_tt.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in "v9 mobilenet_v2 5 2 512" "e4m3 mobilenet_v2 4 3 512" "v5 mobilenet_v2 5 2 512 --v5-ofuf" "vit vit_b16 4 3 64"; do
  set -- $cfg; T=$1; shift
  for v in before after; do
    if [ $v = before ]; then export FP8A_LIB_PATH=$PWD/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
    timeout -k 10 300 python bench.py --arch $1 --expo-width $2 --mant-width $3 --batch $4 $5 --no-cpu-baseline --no-graph \
        > $OUT/${T}_$v.json 2> $OUT/${T}_$v.err || { tail -3 $OUT/${T}_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/${T}_$v.json')); print('$T $v', round(d['value'],1), round(d['roofline']['op_avg_ms'],4))"
  done
done
unset FP8A_LIB_PATH
