#!/bin/bash
# Round 5 (d3): the bordered A pre-pass (padded convolutions) with 4 chunks in flight per thread:
# tests, then interleaved eager A/B lines against _ab/lib_before.so on ResNet-18 and MobileNetV2.
set -o pipefail
OUT=gpurun_out/r05d3; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f8mx.py tests/test_gpu_qin.py \
    tests/test_gpu_chain.py tests/test_gpu_tt.py tests/test_gpu_f8_e5m2.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in "r18 resnet18 4 3 1024" "e4m3 mobilenet_v2 4 3 512"; do
  set -- $cfg; T=$1; shift
  for rep in 1 2; do
    for v in before after; do
      if [ $v = before ]; then export FP8A_LIB_PATH=$PWD/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
      timeout -k 10 300 python bench.py --arch $1 --expo-width $2 --mant-width $3 --batch $4 --no-cpu-baseline --no-graph \
          > $OUT/${T}_${v}_$rep.json 2> $OUT/${T}_${v}_$rep.err || { tail -3 $OUT/${T}_${v}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${T}_${v}_$rep.json')); print('$T $v $rep', round(d['value'],1), round(d['roofline']['op_avg_ms'],4))"
    done
  done
done
unset FP8A_LIB_PATH
