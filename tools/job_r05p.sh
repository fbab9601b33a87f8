#!/bin/bash
# Round 5, step p: bisect the E3M4 layer-set regression across round-4 trees (_bis/<commit>).
set -o pipefail
OUT=gpurun_out/r05p; mkdir -p $OUT
for c in r3 cae4a15 c594aec c5a9530 87b5387 7270225 edd8539; do
  (cd _bis/$c && timeout -k 10 300 python tools/gemm_bench.py --mode w2u --reps 5 > ../../$OUT/$c.log 2>&1) || { tail -5 $OUT/$c.log; exit 1; }
  echo "$c $(tail -1 $OUT/$c.log)"
done
timeout -k 10 300 python tools/gemm_bench.py --mode w2u --reps 5 > $OUT/now.log 2>&1 && echo "now $(tail -1 $OUT/now.log)"
