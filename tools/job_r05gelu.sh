#!/bin/bash
# Round 5 (gelu): the GELU tail of fp8a_matmul_block (post_act 2: ViT's dense + GELU + quantize in one
# launch) -- its tests and the ViT-B/16 line against the previous library (_ab/lib_before.so);
# then the f16 tile-table kernel on short-K E3M4 launches (FP8A_TT16_MINK=64 vs the default 256)
# on ResNet-50.
set -o pipefail
OUT=gpurun_out/r05gelu; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_linear_block.py \
    tests/test_gpu_vit.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in before after; do
  if [ $v = before ]; then export FP8A_LIB_PATH=$PWD/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
  timeout -k 10 300 python bench.py --arch vit_b16 --batch 64 --no-cpu-baseline > $OUT/vit_$v.json 2> $OUT/vit_$v.err \
      || { tail -3 $OUT/vit_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/vit_$v.json')); print('vit $v', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1))"
done
unset FP8A_LIB_PATH
for mk in 256 64; do
  FP8A_TT16_MINK=$mk timeout -k 10 400 python bench.py --arch resnet50 --expo-width 3 --mant-width 4 --batch 512 \
      --no-cpu-baseline > $OUT/r50_e3m4_mink$mk.json 2> $OUT/r50_e3m4_mink$mk.err || { tail -3 $OUT/r50_e3m4_mink$mk.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/r50_e3m4_mink$mk.json')); print('r50 e3m4 mink $mk', round(d['value'],1), d.get('gemm_paths'))"
done
