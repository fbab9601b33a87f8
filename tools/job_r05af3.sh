#!/bin/bash
# Round 5 (af3): the stride-aware af32 threshold (max column tiles x sh x sw) against the plain
# maxct 1 library (_ab/lib_before.so): chain / shape tests, then interleaved graph-timed ResNet-18
# and ResNet-50 E4M3 lines.
set -o pipefail
OUT=gpurun_out/r05af3; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_xm_shapes.py tests/test_gpu_chain.py \
    tests/test_gpu_f8mx.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in "r18 resnet18 1024" "r50 resnet50 512"; do
  set -- $cfg
  for rep in 1 2; do
    for v in before after; do
      if [ $v = before ]; then export FP8A_LIB_PATH=$PWD/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
      timeout -k 10 300 python bench.py --arch $2 --batch $3 --no-cpu-baseline > $OUT/$1_${v}_$rep.json 2> $OUT/$1_${v}_$rep.err \
          || { tail -3 $OUT/$1_${v}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$1_${v}_$rep.json')); print('$1 $v $rep', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1))"
    done
  done
done
unset FP8A_LIB_PATH
