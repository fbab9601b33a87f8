#!/bin/bash
# Round 4: E5M2 top binade on the matrix core (halved MX blocks) + the A-side scale layout probe.
set -o pipefail
OUT=gpurun_out/e5m2b; mkdir -p $OUT
timeout -k 5 60 ./tools/bin_scale_a > $OUT/scale_a.txt 2>&1 || exit $?
cat $OUT/scale_a.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f8_e5m2.py \
    tests/test_gpu_f8.py tests/test_gpu_mbv2_layers.py > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --no-cpu-baseline > $OUT/bench_mb_v9.json 2> $OUT/bench_mb_v9.err || exit $?
cut -c1-200 $OUT/bench_mb_v9.json
python -c "import json; d=json.load(open('$OUT/bench_mb_v9.json')); print(d.get('fallback'))"
timeout -k 10 300 python bench.py --arch resnet50 --expo-width 5 --mant-width 2 --no-cpu-baseline > $OUT/bench_r50.json 2> $OUT/bench_r50.err || exit $?
cut -c1-200 $OUT/bench_r50.json
python -c "import json; d=json.load(open('$OUT/bench_r50.json')); print(d.get('fallback'))"
