#!/bin/bash
# Round 4: MobileNetV2 E5M2 (BASELINE config 3) -- v9 (the literal config: OF/UF flags are no-ops
# in v9) and the v5 OFUF reinterpretation: bench lines + kernel traces with per-kernel breakdowns.
set -o pipefail
OUT=gpurun_out/mb_e5m2; mkdir -p $OUT
timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --no-cpu-baseline > $OUT/bench_v9.json 2> $OUT/bench_v9.err || exit $?
cut -c1-200 $OUT/bench_v9.json
timeout -k 10 300 python bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --v5-ofuf --no-cpu-baseline > $OUT/bench_v5.json 2> $OUT/bench_v5.err || exit $?
cut -c1-200 $OUT/bench_v5.json
R=$(pwd)
for mode in v9 v5; do
  extra=""; [ $mode = v5 ] && extra="--v5-ofuf"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_$mode -o run -- \
      python $R/bench.py --arch mobilenet_v2 --expo-width 5 --mant-width 2 --batch 512 --no-cpu-baseline --steps 3 --warmup 1 $extra > $R/$OUT/trace_$mode.log 2>&1 ) || exit $?
  python tools/trace_breakdown.py $(ls $OUT/trace_$mode/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_$mode.txt | sed -n 2,14p
done
