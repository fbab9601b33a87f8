#!/bin/bash
# Round-5 last check on the final tree: the whole GPU suite, smoke(), the default bench line, and
# the MobileNetV2 E4M3 evidence (tools/job_evidence_r05.sh).
set -o pipefail
OUT=gpurun_out/final5c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', round(d['value'],1), d['roofline']['frac'])"
bash tools/job_evidence_r05.sh mbv2_e4m3 > $OUT/evidence.log 2>&1 || { tail -5 $OUT/evidence.log; exit 1; }
grep -E "^mbv2" $OUT/evidence.log
