#!/bin/bash
# GPU pass for the fused linear / ViT work (run from the repo root via gpurun):
#   new GPU tests -> ViT-B/16 bench line -> rocprofv3 kernel trace of the ViT bench
#   -> operand-exponent statistics of the ResNet-18 layers (tools/unsafe_stats.py)
set -o pipefail
OUT=gpurun_out/${1:-vit}
mkdir -p $OUT
R=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear_block.py tests/test_gpu_vit.py tests/test_gpu_operator.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --arch vit_b16 > $OUT/bench_vit.json 2> $OUT/bench_vit.err || exit $?
cat $OUT/bench_vit.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/vit_trace -o run -- \
    python $R/bench.py --arch vit_b16 --steps 3 --warmup 1 --no-cpu-baseline > $R/$OUT/vit_trace.log 2>&1 || exit $?
cd $R
head -25 $OUT/vit_trace/*kernel_stats.csv
timeout -k 10 400 python -u tools/unsafe_stats.py --arch resnet18 --out $OUT/unsafe_r18.json > $OUT/unsafe.log 2>&1
echo "unsafe_stats rc=$?"
