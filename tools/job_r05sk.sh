#!/bin/bash
# Round 5 (sk): split-K reduction with 32-bit index divisions: split-K / chain tests, then
# interleaved graph-timed ResNet-18 / ViT lines against _ab/lib_before.so, and a kernel trace of
# the ResNet-18 line for the reduction's time.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r05sk; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f8mx.py tests/test_gpu_chain.py \
    tests/test_gpu_parity.py tests/test_gpu_linear_block.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for cfg in "r18 resnet18 1024" "vit vit_b16 64"; do
  set -- $cfg
  for rep in 1 2; do
    for v in before after; do
      if [ $v = before ]; then export FP8A_LIB_PATH=$R/_ab/lib_before.so; else unset FP8A_LIB_PATH; fi
      timeout -k 10 300 python bench.py --arch $2 --batch $3 --no-cpu-baseline > $OUT/$1_${v}_$rep.json 2> $OUT/$1_${v}_$rep.err \
          || { tail -3 $OUT/$1_${v}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/$1_${v}_$rep.json')); print('$1 $v $rep', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1))"
    done
  done
done
unset FP8A_LIB_PATH
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- \
    python $R/bench.py --no-cpu-baseline --no-graph --steps 3 --warmup 1 > $OUT/trace.log 2>&1 || exit 1
cd $R && python tools/trace_breakdown.py $(ls $OUT/trace/*kernel_trace.csv) --forwards 5:3 --out $OUT/breakdown.txt > /dev/null && sed -n 1,12p $OUT/breakdown.txt
