#!/bin/bash
# The one parametrised GPU-job runner (replaces the per-round tools/job_*.sh one-offs, which stay in
# git history).  Every step runs under its own time limit; the first failing step ends the job (no
# GPU step after a fault, an abort or a time limit).  Output under gpurun_out/<job>/.
#
#   bash tools/gpu_job.sh <job> <step> [<step> ...]
# steps (each one word; ':' separates its arguments):
#   tests[:<pytest -k expr>]    python -m pytest tests -m gpu (optionally -k EXPR), 120 s per test
#   smoke                       __graft_entry__.smoke()
#   bench:<name>[:<args>]       bench.py <args with ',' for spaces> -> <job>/bench_<name>.json
#   evidence:<tag>              kernel trace + PMC passes + summary + bench line of one configuration
#                               (tools/profile_config.sh; tags as in tools/evidence_specs.txt)
#   py:<script>[:<args>]        python <script> <args with ',' for spaces> (probes under tools/)
set -o pipefail
JOB=$1; shift
[ -n "$JOB" ] || { echo "usage: gpu_job.sh <job> <step>..." >&2; exit 2; }
OUT=gpurun_out/$JOB; mkdir -p $OUT
ROUND=${FP8A_ROUND:-r06}

spec() {  # evidence tag -> "kernel arch E M batch [bench args]"
  awk -v t="$1" '$1 == t { $1 = ""; print substr($0, 2) }' tools/evidence_specs.txt
}

for step in "$@"; do
  IFS=':' read -r kind a1 a2 <<< "$step"
  case $kind in
    tests)
      K=(); [ -n "$a1" ] && K=(-k "$a1")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -q -x "${K[@]}" --timeout 600 --timeout-method thread \
          > $OUT/tests.log 2>&1
      rc=$?; grep -E "^FAILED|^ERROR|passed|failed" $OUT/tests.log | tail -25
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${a2//,/ } > $OUT/bench_$a1.json 2> $OUT/bench_$a1.err \
          || { tail -8 $OUT/bench_$a1.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/bench_$a1.json')); r=d.get('roofline') or {}; \
print('$a1', round(d['value'],1), {k: r.get(k) for k in ('frac','op_frac','hbm_gbs','valu_busy')}, \
d.get('fallback', {}).get('exact_units'), (d.get('hip_graph') or {}).get('captured'))" ;;
    evidence)
      set -- $(spec $a1); [ -n "$1" ] || { echo "unknown evidence tag $a1" >&2; exit 2; }
      KN=$1; ARCH=$2; E=$3; M=$4; B=$5; shift 5; EXTRA="$*"
      bash tools/profile_config.sh ${JOB}_$a1 $KN $ARCH $E $M $B $EXTRA > $OUT/$a1.prof.log 2>&1 || { tail -5 $OUT/$a1.prof.log; exit 1; }
      cp gpurun_out/${JOB}_$a1/pmc.json $OUT/pmc_${ROUND}_$a1.json
      cp gpurun_out/${JOB}_$a1/summary.txt $OUT/rocprof_${ROUND}_${a1}_summary.txt
      python tools/trace_breakdown.py $(ls gpurun_out/${JOB}_$a1/trace/*kernel_trace.csv) --forwards 5:3 \
          --out $OUT/rocprof_${ROUND}_${a1}_breakdown.txt > /dev/null || exit 1
      sed -n 2,9p $OUT/rocprof_${ROUND}_${a1}_breakdown.txt
      timeout -k 10 600 python bench.py --arch $ARCH --expo-width $E --mant-width $M --batch $B $EXTRA \
          > $OUT/bench_${ROUND}_${a1}_ev.json 2> $OUT/bench_${ROUND}_$a1.err || { tail -3 $OUT/bench_${ROUND}_$a1.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/bench_${ROUND}_${a1}_ev.json')); r=d.get('roofline') or {}; \
print('$a1', round(d['value'],1), {k: r.get(k) for k in ('frac','op_frac','hbm_gbs','valu_busy')})" ;;
    py)
      timeout -k 10 600 python -u $a1 ${a2//,/ } > $OUT/$(basename $a1 .py).log 2>&1 || { tail -20 $OUT/$(basename $a1 .py).log; exit 1; }
      tail -5 $OUT/$(basename $a1 .py).log ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
