#!/bin/bash
# Round 5, step i: fq_apply_fast in the streaming passes only; quad depthwise. Tests, config-1 per
# depthwise form, MobileNetV2 E4M3, ResNet-18 headline.
set -o pipefail
OUT=gpurun_out/r05i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_grouped_conv.py tests/test_gpu_qin.py tests/test_gpu_mbv2_layers.py tests/test_gpu_tbx.py \
    tests/test_gpu_chain.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for dw in 1 2 1 2; do
  FP8A_DW3=$dw timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-approx --no-cpu-baseline \
      > $OUT/c1_dw$dw.json 2> $OUT/c1_dw$dw.err || { tail -5 $OUT/c1_dw$dw.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c1_dw$dw.json')); print('c1 dw3=$dw', round(d['value'],1), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-cpu-baseline > $OUT/mb_e4m3.json 2> $OUT/mb_e4m3.err || exit 1
python -c "import json; d=json.load(open('$OUT/mb_e4m3.json')); print('mbv2 e4m3', round(d['value'],1))"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/r18.json 2> $OUT/r18.err || exit 1
python -c "import json; d=json.load(open('$OUT/r18.json')); print('r18', round(d['value'],1), d['roofline']['frac'])"
