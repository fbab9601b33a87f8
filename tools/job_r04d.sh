#!/bin/bash
# Round 4: E5M2 depthwise on the table form, the pre-checked extreme records: tests, bench lines,
# MobileNetV2 E5M2 trace breakdown.
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
R=$(pwd)
TESTS=${TESTS:-"tests/test_gpu_tbx.py tests/test_gpu_mbv2_layers.py tests/test_gpu_f8_e5m2.py
    tests/test_gpu_chain.py tests/test_gpu_model.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "mb_e5m2:--arch mobilenet_v2 --expo-width 5 --mant-width 2" "r50_e5m2:--arch resnet50 --expo-width 5 --mant-width 2" \
            "r18:--arch resnet18"; do
  tag=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit $?
  cut -c1-150 $OUT/bench_$tag.json
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_mb -o run -- \
    python $R/bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_mb.log 2>&1 ) || exit $?
python tools/trace_breakdown.py $(ls $OUT/trace_mb/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_mb_e5m2.txt | sed -n 2,14p
