#!/bin/bash
set -o pipefail
OUT=gpurun_out/dwg; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dwx.py -m gpu -q --maxfail 10 --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="python bench.py --arch mobilenet_v2 --steps 5 --warmup 2 --no-cpu-baseline"
for m in 0 3; do
    FP8A_DW=$m timeout -k 10 300 $B > $OUT/mb_dw$m.json 2> $OUT/mb_dw$m.err || exit $?
    python -c "import json; d=json.load(open('$OUT/mb_dw$m.json')); print('dw$m', round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['approx_macs_per_s']/1e12,2), d['fallback']['exact_launches'], d['fallback']['tb_launches'])"
done
