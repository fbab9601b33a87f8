#!/bin/bash
# Round-end re-verification after the af32_maxct / v5-depthwise changes: GPU suite, smoke, headline,
# MobileNetV2, ResNet-50 E4M3 lines.
set -o pipefail
OUT=gpurun_out/final2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_r18.json 2> $OUT/bench_r18.err || exit $?
cut -c1-300 $OUT/bench_r18.json
for a in mobilenet_v2 resnet50; do
    timeout -k 10 300 python bench.py --arch $a --no-cpu-baseline > $OUT/bench_$a.json 2> $OUT/bench_$a.err || exit $?
    python -c "import json; d=json.load(open('$OUT/bench_$a.json')); print('$a', round(d['value'],1), d['roofline']['frac'], d['roofline']['traffic'])"
done
