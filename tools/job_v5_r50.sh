#!/bin/bash
# v5 depthwise direct launch: tests + the config-3 line; ResNet-50 E4M3 in-kernel A decode A/B.
set -o pipefail
OUT=gpurun_out/v5r50; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_mbv2_layers.py tests/test_gpu_v5.py tests/test_gpu_tbx.py -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --v5-ofuf --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit $?
python -c "import json; d=json.load(open('$OUT/c3.json')); print('c3', round(d['value'],1), d['ms_per_step'])"
for m in 0 2 4; do
    FP8A_AF32_MAXCT=$m timeout -k 10 300 python bench.py --arch resnet50 --no-cpu-baseline > $OUT/r50_ct$m.json 2> $OUT/r50_ct$m.err || exit $?
    python -c "import json; d=json.load(open('$OUT/r50_ct$m.json')); print('r50 maxct $m', round(d['value'],1), d['ms_per_step'])"
done
