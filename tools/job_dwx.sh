#!/bin/bash
# depthwise band kernel: parity tests, then MobileNetV2 E4M3 bench + kernel-trace breakdown
set -o pipefail
OUT=gpurun_out/dwx; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dwx.py tests/test_gpu_tbx.py tests/test_gpu_mbv2_layers.py tests/test_gpu_model.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --arch mobilenet_v2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_mb.json 2> $OUT/bench_mb.err || exit $?
cat $OUT/bench_mb.json
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace -o run -- python $R/bench.py --arch mobilenet_v2 --steps 3 --warmup 1 --no-cpu-baseline > $R/$OUT/trace.log 2>&1 || exit $?
cd $R && python tools/trace_breakdown.py $(ls $OUT/trace/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown.txt | head -20
