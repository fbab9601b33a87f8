#!/bin/bash
# Round 5, step n: the E3M4 / E2M5 layer set, round-3 tree (_r3: its own package and library) vs now.
set -o pipefail
OUT=gpurun_out/r05n; mkdir -p $OUT
for m in w2u lut; do
  (cd _r3 && timeout -k 10 300 python tools/gemm_bench.py --mode $m --reps 5 > ../$OUT/r3_$m.log 2>&1) || { tail -5 $OUT/r3_$m.log; exit 1; }
  timeout -k 10 300 python tools/gemm_bench.py --mode $m --reps 5 > $OUT/now_$m.log 2>&1 || exit 1
  echo "$m r3  $(tail -1 $OUT/r3_$m.log)"
  echo "$m now $(tail -1 $OUT/now_$m.log)"
done
