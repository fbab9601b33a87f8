#!/bin/bash
# Round 4: own-output-quantizer fusion + table-form hand-off: tests, bench lines, MobileNetV2 trace.
set -o pipefail
OUT=gpurun_out/r04h; mkdir -p $OUT
R=$(pwd)
TESTS=${TESTS:-"tests/test_gpu_model.py tests/test_gpu_mbv2_layers.py tests/test_gpu_chain.py tests/test_gpu_tbx.py
    tests/test_gpu_fused_bn.py tests/test_gpu_v5.py tests/test_gpu_qin.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "mb_e4m3:--arch mobilenet_v2" "mb_e5m2_v9:--arch mobilenet_v2 --expo-width 5 --mant-width 2" \
            "mb_e5m2_v5:--arch mobilenet_v2 --expo-width 5 --mant-width 2 --v5-ofuf" "r18:--arch resnet18"; do
  tag=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit $?
  cut -c1-140 $OUT/bench_$tag.json
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_mb -o run -- \
    python $R/bench.py --arch mobilenet_v2 --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_mb.log 2>&1 ) || exit $?
python tools/trace_breakdown.py $(ls $OUT/trace_mb/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_mb_e4m3.txt | sed -n 2,14p
