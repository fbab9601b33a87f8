#!/bin/bash
# Round 5 (vd): the matrix-A pre-pass at one chunk per thread (ViT's token rows) against four
# (_ab/lib_before.so): interleaved eager ViT-B/16 lines.
set -o pipefail
OUT=gpurun_out/r05vd; mkdir -p $OUT
for rep in 1 2; do
  for v in before after; do
    if [ $v = before ]; then export FP8A_LIB_PATH=$PWD/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
    timeout -k 10 300 python bench.py --arch vit_b16 --batch 64 --steps 10 --no-cpu-baseline --no-graph > $OUT/vit_${v}_$rep.json \
        2> $OUT/vit_${v}_$rep.err || { tail -3 $OUT/vit_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/vit_${v}_$rep.json')); print('vit $v $rep', round(d['value'],1), round(d['roofline']['op_avg_ms'],4))"
  done
done
