#!/bin/bash
# Round 5 (af2): ResNet-18 (the headline) with af32_maxct 1 (default) vs 3, interleaved, graph-timed.
set -o pipefail
OUT=gpurun_out/r05af2; mkdir -p $OUT
for rep in 1 2 3; do
  for mc in 1 3; do
    FP8A_AF32_MAXCT=$mc timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/r18_mc${mc}_$rep.json 2> $OUT/r18_mc${mc}_$rep.err \
        || { tail -3 $OUT/r18_mc${mc}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/r18_mc${mc}_$rep.json')); print('r18 maxct $mc $rep', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1))"
  done
done
