#!/bin/bash
# Round-end verification on one box: GPU suite, smoke, headline bench (with CPU baseline), the
# MobileNetV2 line, and rocprofv3 evidence (trace + FETCH / WRITE) for both.
set -o pipefail
OUT=gpurun_out/final; mkdir -p $OUT
# depthwise forms first: identity tests, then the MobileNetV2 A/B (word-image gather vs fp32 gather)
bash tools/job_dwg_ab.sh || exit $?
# the faster depthwise form for the lines below (the A/B picks the default committed afterwards)
export FP8A_DW=$(python -c "import json; v={m: json.load(open(f'gpurun_out/dwg/mb_dw{m}.json'))['value'] for m in (0, 2)}; print(max(v, key=v.get))")
echo "FP8A_DW=$FP8A_DW"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_r18.json 2> $OUT/bench_r18.err || exit $?
cut -c1-400 $OUT/bench_r18.json
timeout -k 10 300 python bench.py --arch mobilenet_v2 --no-cpu-baseline > $OUT/bench_mb.json 2> $OUT/bench_mb.err || exit $?
cut -c1-300 $OUT/bench_mb.json
bash tools/profile_config.sh r18_e4m3_r3 gemm_f8mx_kernel resnet18 4 3 512 > $OUT/prof_r18.log 2>&1 || { tail $OUT/prof_r18.log; exit 1; }
python tools/trace_breakdown.py $(ls gpurun_out/r18_e4m3_r3/trace/*kernel_trace.csv) --forwards 5:3 --out gpurun_out/r18_e4m3_r3/breakdown.txt | sed -n 2,10p
bash tools/profile_config.sh mb_e4m3_r3 gemm_f8mx_kernel mobilenet_v2 4 3 512 > $OUT/prof_mb.log 2>&1 || { tail $OUT/prof_mb.log; exit 1; }
python tools/trace_breakdown.py $(ls gpurun_out/mb_e4m3_r3/trace/*kernel_trace.csv) --forwards 5:3 --out gpurun_out/mb_e4m3_r3/breakdown.txt | sed -n 2,12p
