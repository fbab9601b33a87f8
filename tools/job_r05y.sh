#!/bin/bash
# Round 5 (y): bench.py's HIP-graph mode (the forward captured once, each timed step one replay)
# on every configuration: the line's value (replays) against its hip_graph.eager_images_per_s (the
# same steps eager, right after), and the capture's bitwise check against an eager forward.
set -o pipefail
OUT=gpurun_out/r05y; mkdir -p $OUT
for cfg in "c1 mobilenet_v2 4 3 512 --no-approx" "mbv2_e4m3 mobilenet_v2 4 3 512" "c3v5 mobilenet_v2 5 2 512 --v5-ofuf" \
           "c3v9 mobilenet_v2 5 2 512" "vit vit_b16 4 3 64" "r18 resnet18 4 3 1024"; do
  set -- $cfg
  T=$1; shift
  timeout -k 10 300 python bench.py --arch $1 --expo-width $2 --mant-width $3 --batch $4 $5 --no-cpu-baseline \
      > $OUT/$T.json 2> $OUT/$T.err || { tail -5 $OUT/$T.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$T.json')); g=d.get('hip_graph') or {}; print('$T', round(d['value'],1), 'eager', round(g.get('eager_images_per_s', 0),1), g.get('captured'), g.get('error'))"
done
