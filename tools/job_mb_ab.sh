#!/bin/bash
# MobileNetV2 E4M3 A/B: the depthwise and GEMM schedules of round 3 against round 2's, after the
# affected parity tests.  Usage: bash tools/job_mb_ab.sh <tag>
set -o pipefail
TAG=${1:-mbab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dwx.py tests/test_gpu_tbx.py tests/test_gpu_xm_shapes.py tests/test_gpu_mbv2_layers.py -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="python bench.py --arch mobilenet_v2 --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $B > $OUT/mb_default.json 2> $OUT/mb_default.err || exit $?
timeout -k 10 300 $B > $OUT/mb_nodwx.json 2> $OUT/mb_nodwx.err || exit $?
FP8A_NO_DWX=1 FP8A_XM_NCG=4 FP8A_AF32_MAXCT=0 timeout -k 10 300 $B > $OUT/mb_r2sched.json 2> $OUT/mb_r2sched.err || exit $?
for f in default nodwx r2sched; do python -c "import json,sys; d=json.load(open('$OUT/mb_$f.json')); print('$f', round(d['value'],1), round(d['ms_per_step'],3), d['roofline']['approx_macs_per_s']/1e12, d['fallback']['exact_launches'])"; done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/trace -o run -- python $R/bench.py --arch mobilenet_v2 --steps 3 --warmup 1 --no-cpu-baseline > $R/$OUT/trace.log 2>&1 || exit $?
cd $R && python tools/trace_breakdown.py $(ls $OUT/trace/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown.txt | head -16
