#!/bin/bash
# Round 5 (f2): af32_maxct default 1 -- the whole GPU suite, smoke(), then graph-timed lines on the
# configurations it touches (MobileNetV2 E4M3, config 3 v9 / v5, ResNet-18, ResNet-50 E4M3 / E5M2).
set -o pipefail
OUT=gpurun_out/r05f2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for cfg in "mbv2_e4m3 mobilenet_v2 4 3 512" "v9 mobilenet_v2 5 2 512" "v5 mobilenet_v2 5 2 512 --v5-ofuf" "r18 resnet18 4 3 1024" \
           "r50_e4m3 resnet50 4 3 512" "r50_e5m2 resnet50 5 2 512"; do
  set -- $cfg; T=$1; shift
  timeout -k 10 300 python bench.py --arch $1 --expo-width $2 --mant-width $3 --batch $4 $5 --no-cpu-baseline > $OUT/$T.json \
      2> $OUT/$T.err || { tail -3 $OUT/$T.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$T.json')); print('$T', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1))"
done
