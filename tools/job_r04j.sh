#!/bin/bash
# Round 4: LDS-staged depthwise kernels (exact dn_dw3_kernel, table-form conv_tbs_kernel) and the
# HIP AvgPool2d: tests, MobileNetV2 bench A/B lines, traces.
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
R=$(pwd)
TESTS=${TESTS:-"tests/test_gpu_tbx.py tests/test_gpu_grouped_conv.py tests/test_gpu_pool.py tests/test_gpu_mbv2_layers.py
    tests/test_gpu_model.py tests/test_gpu_chain.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for spec in "mb_e4m3_tbs1:FP8A_TBS=1:--arch mobilenet_v2" "mb_e4m3_tbs0:FP8A_TBS=0:--arch mobilenet_v2" \
            "mb_e5m2_v9:FP8A_TBS=1:--arch mobilenet_v2 --expo-width 5 --mant-width 2" \
            "c1_dw3_1:FP8A_DW3=1:--arch mobilenet_v2 --no-approx" "c1_dw3_0:FP8A_DW3=0:--arch mobilenet_v2 --no-approx"; do
  tag=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; a=${rest#*:}
  env $envs timeout -k 10 300 python bench.py $a --no-cpu-baseline > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit $?
  echo "$tag $(cut -c1-120 $OUT/bench_$tag.json)"
done
for spec in "mb:--arch mobilenet_v2" "c1:--arch mobilenet_v2 --no-approx"; do
  tag=${spec%%:*}; a=${spec#*:}
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_$tag -o run -- \
      python $R/bench.py $a --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_$tag.log 2>&1 ) || exit $?
  python tools/trace_breakdown.py $(ls $OUT/trace_$tag/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_$tag.txt | sed -n 2,12p
done
