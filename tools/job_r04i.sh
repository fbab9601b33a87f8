#!/bin/bash
# Round 4: the LDS-staged exact depthwise (dn_dw3_kernel): tests, config-1 bench A/B (FP8A_DW3=1 / 0),
# trace breakdown.
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
R=$(pwd)
TESTS=${TESTS:-"tests/test_gpu_grouped_conv.py tests/test_gpu_pool.py tests/test_gpu_dense.py tests/test_gpu_model.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
  FP8A_DW3=$f timeout -k 10 300 python bench.py --arch mobilenet_v2 --no-approx --no-cpu-baseline > $OUT/bench_c1_dw3$f.json 2> $OUT/bench_c1_dw3$f.err || exit $?
  cut -c1-140 $OUT/bench_c1_dw3$f.json
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_c1 -o run -- \
    python $R/bench.py --arch mobilenet_v2 --no-approx --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_c1.log 2>&1 ) || exit $?
python tools/trace_breakdown.py $(ls $OUT/trace_c1/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_c1.txt | sed -n 2,16p
