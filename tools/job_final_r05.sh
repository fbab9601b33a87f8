#!/bin/bash
# Round-5 verification on one box: the whole GPU suite, smoke(), then the ViT-B/16 evidence
# (kernel trace, PMC passes, bench line) of tools/job_evidence_r05.sh.
set -o pipefail
OUT=gpurun_out/final5; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
bash tools/job_evidence_r05.sh c4_vit_b16 > $OUT/evidence.log 2>&1 || { tail -5 $OUT/evidence.log; exit 1; }
grep -E "^c4" $OUT/evidence.log
