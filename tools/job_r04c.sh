#!/bin/bash
# Round 4: E5M2 tile-level routing to the halved-block form, the exact grouped convolution
# (config 1 without torch convolutions): tests, bench lines, config-1 trace breakdown.
set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT
R=$(pwd)
timeout -k 5 60 ./tools/bin_mfma_bf16_denorm > $OUT/bf16_denorm.txt 2>&1 || exit $?
cat $OUT/bf16_denorm.txt
TESTS=${TESTS:-"tests/test_gpu_grouped_conv.py tests/test_gpu_model.py tests/test_gpu_f8_e5m2.py tests/test_gpu_f8.py
    tests/test_gpu_mbv2_layers.py tests/test_gpu_model_formats.py tests/test_gpu_dense.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "r50_e5m2:--arch resnet50 --expo-width 5 --mant-width 2" "mb_e5m2:--arch mobilenet_v2 --expo-width 5 --mant-width 2" \
            "c1_mb_noapprox:--arch mobilenet_v2 --no-approx"; do
  tag=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit $?
  cut -c1-180 $OUT/bench_$tag.json
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_c1 -o run -- \
    python $R/bench.py --arch mobilenet_v2 --no-approx --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_c1.log 2>&1 ) || exit $?
python tools/trace_breakdown.py $(ls $OUT/trace_c1/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_c1.txt | sed -n 2,14p
