#!/bin/bash
# Round-4 verification on one box: the whole GPU suite, smoke(), the headline bench line (with its
# CPU baseline) and its rocprofv3 kernel trace + stats summary.
set -o pipefail
OUT=gpurun_out/final4; mkdir -p $OUT
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_r18.json 2> $OUT/bench_r18.err || exit $?
cut -c1-300 $OUT/bench_r18.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace_r18 -o run -- \
    python $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/$OUT/trace_r18.log 2>&1 ) || exit $?
python tools/trace_breakdown.py $(ls $OUT/trace_r18/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_r18.txt | sed -n 2,10p
