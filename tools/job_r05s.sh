#!/bin/bash
# Round 5, step s: split-K heuristic A/B (FP8A_SPLITK=1 forces one split) on ViT-B/16, ResNet-18, ResNet-50 E4M3.
set -o pipefail
OUT=gpurun_out/r05s; mkdir -p $OUT
run() {  # tag, bench args, env
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline $args > $OUT/$tag.json 2> $OUT/$tag.err || { tail -3 $OUT/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); r=d['roofline']; print('$tag', round(d['value'],1), round(r.get('kernel_avg_ms') or 0,4), round(r.get('op_avg_ms') or 0,4))"
}
for r in 1 2; do
  run vit_def "--arch vit_b16 --batch 64" FP8A_X=1 || exit 1
  run vit_s1 "--arch vit_b16 --batch 64" FP8A_SPLITK=1 || exit 1
done
run r18_def "" FP8A_X=1 || exit 1
run r18_s1 "" FP8A_SPLITK=1 || exit 1
run r50_def "--arch resnet50 --batch 512" FP8A_X=1 || exit 1
run r50_s1 "--arch resnet50 --batch 512" FP8A_SPLITK=1 || exit 1
