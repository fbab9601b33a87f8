#!/bin/bash
# GPU suite, then the headline + MobileNetV2 E4M3 bench lines and a MobileNetV2 kernel-trace breakdown.
# Usage: bash tools/job_mb.sh <tag> [pytest selection]
set -o pipefail
TAG=${1:-mb}; SEL=${2:-tests}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $SEL -m gpu -q --maxfail 20 --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
# (assertion failures still allow the benches; a crash / hang / timeout does not)
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --arch mobilenet_v2 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_mb.json 2> $OUT/bench_mb.err || exit $?
cat $OUT/bench_mb.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_r18.json 2> $OUT/bench_r18.err || exit $?
cat $OUT/bench_r18.json
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace -o run -- python $R/bench.py --arch mobilenet_v2 --steps 3 --warmup 1 --no-cpu-baseline > $R/$OUT/trace.log 2>&1 || exit $?
cd $R && python tools/trace_breakdown.py $(ls $OUT/trace/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown.txt | head -24
