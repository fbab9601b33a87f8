#!/bin/bash
# Round 5 (x): the self-cleaning flag arena (no fill per launch) + the flattened A pre-pass:
# new tests, the whole GPU suite, smoke(), then A/B bench lines against the previous library
# (_ab/lib_before.so) on ViT-B/16, MobileNetV2 E4M3 and ResNet-18.
set -o pipefail
OUT=gpurun_out/r05x; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_f8mx.py tests/test_gpu_tbx.py > $OUT/new_tests.log 2>&1 || { tail -30 $OUT/new_tests.log; exit 1; }
tail -1 $OUT/new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for cfg in "vit_b16 4 3 64" "mobilenet_v2 4 3 512" "resnet18 4 3 1024"; do
  set -- $cfg
  for v in before after; do
    if [ $v = before ]; then export FP8A_LIB_PATH=$PWD/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
    timeout -k 10 300 python bench.py --arch $1 --expo-width $2 --mant-width $3 --batch $4 --no-cpu-baseline \
        > $OUT/ab_$1_$v.json 2> $OUT/ab_$1_$v.err || { tail -3 $OUT/ab_$1_$v.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/ab_$1_$v.json')); print('$1 $v', round(d['value'],1), d['ms_per_step'])"
  done
done
unset FP8A_LIB_PATH
