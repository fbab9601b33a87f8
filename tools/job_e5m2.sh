#!/bin/bash
# Round 4: E5M2 on the matrix core -- identity tests, E4M3 regression, ResNet-50 E5M2 bench line.
set -o pipefail
OUT=gpurun_out/e5m2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_f8_e5m2.py \
    tests/test_gpu_f8.py tests/test_gpu_model_formats.py tests/test_gpu_fullsize.py > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --arch resnet50 --expo-width 5 --mant-width 2 --no-cpu-baseline > $OUT/bench_r50_e5m2.json 2> $OUT/bench_r50_e5m2.err || exit $?
cut -c1-300 $OUT/bench_r50_e5m2.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_r18.json 2> $OUT/bench_r18.err || exit $?
cut -c1-300 $OUT/bench_r18.json
