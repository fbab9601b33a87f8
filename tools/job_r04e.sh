#!/bin/bash
# Round 4: the v5 forms on the GPU (word-form depthwise, matrix-core GEMM): tests, the config-3 v5
# bench line, its trace breakdown.
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
R=$(pwd)
TESTS=${TESTS:-"tests/test_gpu_v5.py tests/test_gpu_mbv2_layers.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --v5-ofuf --no-cpu-baseline > $OUT/bench_c3_v5.json 2> $OUT/bench_c3_v5.err || exit $?
cut -c1-150 $OUT/bench_c3_v5.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_v5 -o run -- \
    python $R/bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --v5-ofuf --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_v5.log 2>&1 ) || exit $?
python tools/trace_breakdown.py $(ls $OUT/trace_v5/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_c3_v5.txt | sed -n 2,14p
