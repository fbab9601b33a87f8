#!/bin/bash
# Round 5: verification after a library change -- the GPU suite, smoke(), a short headline bench line.
set -o pipefail
OUT=gpurun_out/${1:-r05b}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 > $OUT/bench_r18.json 2> $OUT/bench_r18.err || exit $?
cut -c1-250 $OUT/bench_r18.json
