#!/bin/bash
# Round 5 (ex): the gated exact kernel's grid capped at 512 blocks: fallback tests, then
# interleaved graph-timed lines against _ab/lib_before.so (MobileNetV2 E4M3, ViT, ResNet-18).
set -o pipefail
OUT=gpurun_out/r05ex; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f8mx.py tests/test_gpu_f8_e5m2.py \
    tests/test_gpu_tt.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in "mbv2 mobilenet_v2 512" "vit vit_b16 64" "r18 resnet18 1024"; do
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
