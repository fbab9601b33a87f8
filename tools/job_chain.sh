#!/bin/bash
# Round 4: word-image hand-off -- identity tests, then ResNet-18 with it on and off (bench lines and
# kernel traces with per-kernel breakdowns), ResNet-50 with it on.
set -o pipefail
OUT=gpurun_out/chain; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chain.py \
    tests/test_gpu_qin.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
R=$(pwd)
for c in 1 0; do
  FP8A_CHAIN=$c timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_r18_chain$c.json 2> $OUT/bench_r18_chain$c.err || exit $?
  cut -c1-160 $OUT/bench_r18_chain$c.json
  ( cd /tmp && export TMPDIR=/tmp && FP8A_CHAIN=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace$c -o run -- \
      python $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace$c.log 2>&1 ) || exit $?
  python tools/trace_breakdown.py $(ls $OUT/trace$c/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown$c.txt | sed -n 2,9p
done
for c in 1 0; do
  FP8A_CHAIN=$c timeout -k 10 300 python bench.py --arch resnet50 --no-cpu-baseline > $OUT/bench_r50_chain$c.json 2> $OUT/bench_r50.err || exit $?
  cut -c1-160 $OUT/bench_r50_chain$c.json
done
