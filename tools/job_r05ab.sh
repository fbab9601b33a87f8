#!/bin/bash
# Round 5: interleaved A/B (before, after, before, after) of the current library against
# _ab/lib_before.so on ViT-B/16 (20 steps) and ResNet-18 (5 steps), graph-timed lines.
set -o pipefail
OUT=gpurun_out/r05ab; mkdir -p $OUT
for cfg in "vit vit_b16 64 20" "r18 resnet18 1024 5"; do
  set -- $cfg
  for rep in 1 2; do
    for v in before after; do
      if [ $v = before ]; then export FP8A_LIB_PATH=$PWD/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
      timeout -k 10 300 python bench.py --arch $2 --batch $3 --steps $4 --no-cpu-baseline > $OUT/$1_${v}_$rep.json \
          2> $OUT/$1_${v}_$rep.err || { tail -3 $OUT/$1_${v}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$1_${v}_$rep.json')); print('$1 $v $rep', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1), round(d['roofline']['kernel_avg_ms'],4))"
    done
  done
done
