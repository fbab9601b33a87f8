#!/bin/bash
# Round 5, step u: split-K model of the matrix-core kernel (its own tiles and rate) vs the 64 x 64
# model (FP8A_SPLITK_MODEL=0); unconditional LDS reads in the staged depthwise kernels.
set -o pipefail
OUT=gpurun_out/r05u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tbx.py tests/test_gpu_grouped_conv.py \
    tests/test_gpu_v5.py tests/test_gpu_xm_shapes.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # tag, bench args, env
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline $args > $OUT/$tag.json 2> $OUT/$tag.err || { tail -3 $OUT/$tag.err; return 1; }
  python -c "import json; d=json.load(open('$OUT/$tag.json')); r=d['roofline']; print('$tag', round(d['value'],1), round(r.get('kernel_avg_ms') or 0,4), (d.get('gemm_paths') or {}))" | cut -c1-150
}
for m in 1 0; do
  run r18_m$m "" FP8A_SPLITK_MODEL=$m || exit 1
  run r50_m$m "--arch resnet50 --batch 512" FP8A_SPLITK_MODEL=$m || exit 1
  run vit_m$m "--arch vit_b16 --batch 64" FP8A_SPLITK_MODEL=$m || exit 1
  run mb_m$m "--arch mobilenet_v2 --batch 512" FP8A_SPLITK_MODEL=$m || exit 1
  run r50e5_m$m "--arch resnet50 --batch 512 --expo-width 5 --mant-width 2" FP8A_SPLITK_MODEL=$m || exit 1
done
run c1 "--arch mobilenet_v2 --batch 512 --no-approx" FP8A_X=1 || exit 1
