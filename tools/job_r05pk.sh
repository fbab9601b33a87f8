#!/bin/bash
# Round 5 (pk): conv_tbsg_kernel's terms in lane pairs on packed fp32 (option tbs_pk): the staged
# forms' bit-identity tests, then interleaved eager lines with FP8A_TBS_PK=0 / 1 on MobileNetV2
# E4M3 and E5M2 v9, and the depthwise layer set.
set -o pipefail
OUT=gpurun_out/r05pk; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_tbx.py \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in "e4m3 mobilenet_v2 4 3 512" "v9 mobilenet_v2 5 2 512"; do
  set -- $cfg; T=$1; shift
  for rep in 1 2; do
    for pk in 0 1; do
      FP8A_TBS_PK=$pk timeout -k 10 300 python bench.py --arch $1 --expo-width $2 --mant-width $3 --batch $4 --no-cpu-baseline --no-graph \
          > $OUT/${T}_pk${pk}_$rep.json 2> $OUT/${T}_pk${pk}_$rep.err || { tail -3 $OUT/${T}_pk${pk}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/${T}_pk${pk}_$rep.json')); print('$T pk$pk $rep', round(d['value'],1))"
    done
  done
done
