#!/bin/bash
# Round 5, step f: config-1 kernel traces with the two depthwise staging forms (FP8A_DW3 = 1 / 2),
# the v5 fused-qin tests, config-3 (v5) evidence.
set -o pipefail
OUT=gpurun_out/r05f; mkdir -p $OUT
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qin.py \
    tests/test_gpu_v5.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for dw in 1 2; do
  (cd /tmp && export TMPDIR=/tmp && FP8A_DW3=$dw timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/c1_dw$dw -o run -- \
      python $R/bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline --steps 3 --warmup 1 \
      > $R/$OUT/c1_dw$dw.log 2>&1) || exit 1
  python tools/trace_breakdown.py $(ls $OUT/c1_dw$dw/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown_c1_dw$dw.txt > /dev/null || exit 1
  sed -n 2,12p $OUT/breakdown_c1_dw$dw.txt
done
bash tools/job_evidence_r05.sh c3_mbv2_e5m2_v5
