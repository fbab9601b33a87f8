#!/bin/bash
# Round 4: two-row depthwise table form (tests, MobileNetV2 E4M3 A/B, trace), and the headline
# kernel's VALU / LDS counters for DESIGN §3k.
set -o pipefail
OUT=gpurun_out/r04f; mkdir -p $OUT
R=$(pwd)
TESTS=${TESTS:-"tests/test_gpu_tbx.py tests/test_gpu_mbv2_layers.py"}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for rw in 2 1; do
  FP8A_TBX_RW=$rw timeout -k 10 300 python bench.py --arch mobilenet_v2 --no-cpu-baseline > $OUT/bench_mb_rw$rw.json 2> $OUT/bench_mb_rw$rw.err || exit $?
  cut -c1-130 $OUT/bench_mb_rw$rw.json
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_mb -o run -- \
    python $R/bench.py --arch mobilenet_v2 --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_mb.log 2>&1 ) || exit $?
python tools/trace_breakdown.py $(ls $OUT/trace_mb/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_mb_e4m3.txt | sed -n 2,12p
timeout -k 10 400 bash tools/pmc_lds.sh l3.c2 base > $OUT/pmc_lds.txt 2>&1 || { tail -5 $OUT/pmc_lds.txt; exit 1; }
cat $OUT/pmc_lds.txt
