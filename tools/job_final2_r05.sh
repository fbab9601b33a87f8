#!/bin/bash
# Round-5 final check: the default bench line exactly as the driver runs it (ResNet-18, CPU baseline
# included), timed; then the whole GPU suite and smoke().
set -o pipefail
OUT=gpurun_out/final5b; mkdir -p $OUT
s=$(date +%s)
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
echo "default bench wall $(( $(date +%s) - s )) s"
python -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['hip_graph'], d['cpu_baseline']['value'], d['roofline']['frac'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
