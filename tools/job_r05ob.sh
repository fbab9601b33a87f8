#!/bin/bash
# Round 5 (ob): the output quantizer's bias written by the gated exact kernel (no one-thread launch
# per fused tail) + the gated depthwise literal kernel capped at 1024 blocks: the fused-tail / chain /
# depthwise tests, then interleaved graph-timed lines against _ab/lib_before.so.
set -o pipefail
OUT=gpurun_out/r05ob; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_linear_block.py tests/test_gpu_chain.py \
    tests/test_gpu_tbx.py tests/test_gpu_qin.py tests/test_gpu_vit.py tests/test_gpu_model.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
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
