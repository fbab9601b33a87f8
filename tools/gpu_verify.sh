#!/bin/bash
# One verification pass on the GPU box (run from the repo root via gpurun):
#   pytest -m gpu -> smoke() -> bench.py (headline) [-> extra bench.py args lines]
# Usage: bash tools/gpu_verify.sh <tag> [pytest selector] ["bench args" ...]
set -o pipefail
TAG=${1:-verify}
SEL=${2:-tests}
shift 2 2>/dev/null
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
i=0
for b in "$@"; do
    timeout -k 10 400 python bench.py $b > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit $?
    cat $OUT/bench_$i.json
    i=$((i+1))
done
