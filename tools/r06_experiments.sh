#!/bin/bash
# Round 6's GPU experiments, one function each (the per-round tools/job_*.sh one-offs of rounds 1-5
# are in git history; routine steps are tools/gpu_job.sh's).  Run from the repo root through the
# GPU runner:  bash tools/r06_experiments.sh <name> ...
#   census      tests of the graph / multi-rank paths, the default bench line, the product census of
#               four workloads (tools/census.py -> profiles/r06_census/)
#   ttband      E2M5 band forms: tt tests + ResNet-50 E2M5 with FP8A_TT_BAND 0 / 1
#   ttband_prof rocprof traces of ResNet-50 E2M5 with the band forms off / on
#   ttxk        E2M5 K-steps per staged tile: lib built with -DTT_XK5=4 (lib/ab/) vs the default
#   dwpmc       SQ / LDS counters of the staged depthwise kernels (tools/pmc_kernel.sh)
#   dwab        staged depthwise A/B: lib/ab/libfp8approx_kyu1.so at several block plans
#   v5ab        v5 / E5M2 v9 depthwise A/B: lib/ab/libfp8approx_v5k1.so
#   tt16ab      E3M4 tile-table sub-stages per staged tile: default (2) vs lib/ab/ ns1 (1) and f7ns1 (F7 form: 1)
#   splitab     split-K choice: the default line and ResNet-50 E4M3 with FP8A_SPLITK unset / 1
#   bdma        gemm_f8mx_kernel's B operand by LDS-DMA (plain instance at 6 waves): f8mx tests, then
#               ResNet-18 / ResNet-50 E4M3 with the default, lib/ab/ w6all (every instance at 6) and nobdma
#   dwops       table-form depthwise with fewer VALU ops per term: tbx / chain tests, then MobileNetV2
#               E4M3 and E5M2 v9 with the default vs lib/ab/libfp8approx_r6base.so (the previous commit)
#   tapt        staged table-form depthwise with per-tap tables (TBSG_TAPT): depthwise / chain / model
#               tests, then MobileNetV2 E4M3 and E5M2 v9 with the default vs lib/ab/libfp8approx_tapt0.so
#   dwemit      depthwise -> 1x1 word-image hand-off (form 0 from conv_tbsg_kernel): chain / depthwise /
#               model tests, then MobileNetV2 E4M3 and E5M2 v9 with the hand-off across blocks
#               (FP8A_MBV2_XCHAIN) on and off
#   multirank   two ranks on one GPU over gloo vs two world-1 runs (logits and FP8 state per rank)
# A/B libraries: python -c "from fp8_quantization_amd import build_native as b; b.build(force=True,
#   out='fp8_quantization_amd/lib/ab/<name>.so', extra=b.EXTRA + ['-D...'])"
set -o pipefail
R=$(pwd)
AB=$R/fp8_quantization_amd/lib/ab

bench_line() {  # out-dir name lib bench-args...
  local O=$1 N=$2 L=$3; shift 3
  FP8A_LIB_PATH=$L timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/$N.json 2> $O/$N.err || { tail -3 $O/$N.err; return 1; }
  python -c "import json; d=json.load(open('$O/$N.json')); print('$N', round(d['value'],1), (d.get('hip_graph') or {}).get('eager_images_per_s'), (d.get('roofline') or {}).get('frac'))"
}

census() {
  bash tools/gpu_job.sh census "tests:multirank or graph" bench:default || return 1
  mkdir -p gpurun_out/census
  for cfg in "resnet50 2 5" "resnet50 3 4" "resnet18 4 3" "mobilenet_v2 4 3"; do
    set -- $cfg
    timeout -k 10 300 python -u tools/census.py --arch $1 --expo-width $2 --mant-width $3 --batch 16 --tiles \
      --out gpurun_out/census/census_$1_e$2m$3.json > gpurun_out/census/census_$1_e$2m$3.txt 2>&1 || return 1
    head -1 gpurun_out/census/census_$1_e$2m$3.txt
  done
}

ttband() {
  local O=gpurun_out/ttb; mkdir -p $O
  bash tools/gpu_job.sh ttb "tests:test_gpu_tt or E2M5" || return 1
  for b in 0 1; do FP8A_TT_BAND=$b bench_line $O r50_e2m5_band$b "" --arch resnet50 --expo-width 2 --mant-width 5 --batch 512 || return 1; done
}

ttband_prof() {
  local O=$R/gpurun_out/ttb2; mkdir -p $O
  for b in 0 1; do
    (cd /tmp && export TMPDIR=/tmp && FP8A_TT_BAND=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/t$b -o run -- \
      python $R/bench.py --arch resnet50 --expo-width 2 --mant-width 5 --batch 512 --no-cpu-baseline --steps 3 --warmup 1 \
      --no-graph > $O/t$b.log 2>&1) || return 1
    python tools/trace_breakdown.py $(ls $O/t$b/*kernel_trace.csv) --forwards 5:3 --out $O/bd$b.txt > /dev/null || return 1
    sed -n 1,8p $O/bd$b.txt
  done
}

ttxk() {
  local O=gpurun_out/ttxk; mkdir -p $O
  FP8A_LIB_PATH=$AB/libfp8approx_xk4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tt.py -q -x --timeout 300 \
    > $O/tests_xk4.log 2>&1 || { tail -5 $O/tests_xk4.log; return 1; }
  timeout -k 10 400 python -u tools/tt_band_layer.py > $O/layers_xk2.log 2>&1 || return 1
  FP8A_LIB_PATH=$AB/libfp8approx_xk4.so timeout -k 10 400 python -u tools/tt_band_layer.py > $O/layers_xk4.log 2>&1 || return 1
  for v in xk2 xk4; do
    L=""; [ $v = xk4 ] && L=$AB/libfp8approx_xk4.so
    bench_line $O bench_$v "$L" --arch resnet50 --expo-width 2 --mant-width 5 --batch 512 || return 1
  done
}

dwpmc() {
  bash tools/pmc_kernel.sh dwpmc_tbsg conv_tbsg_kernel --arch mobilenet_v2 --batch 512 || return 1
  bash tools/pmc_kernel.sh dwpmc_v5ds conv_v5ds_kernel --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 --v5-ofuf || return 1
  bash tools/gpu_job.sh ev6 evidence:mbv2_e4m3_dw
}

dwab() {
  local O=gpurun_out/dwab; mkdir -p $O; local K1=$AB/libfp8approx_kyu1.so
  FP8A_LIB_PATH=$K1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tbx.py -q -x --timeout 300 > $O/tests_k1.log 2>&1 || return 1
  FP8A_DW_TARGET=4096 FP8A_DW_LDS=40960 bench_line $O base "" --arch mobilenet_v2 --batch 512 || return 1
  for t in "4096 40960" "2048 20480" "1024 12288"; do
    set -- $t; FP8A_DW_TARGET=$1 FP8A_DW_LDS=$2 bench_line $O k1_$1 $K1 --arch mobilenet_v2 --batch 512 || return 1
  done
}

v5ab() {
  local O=gpurun_out/v5ab; mkdir -p $O; local K1=$AB/libfp8approx_v5k1.so
  FP8A_LIB_PATH=$K1 timeout -k 10 600 python -u -m pytest tests/test_gpu_v5.py tests/test_gpu_chain.py -q -x --timeout 300 \
    > $O/tests_k1.log 2>&1 || return 1
  for v in base k1; do
    L=""; [ $v = k1 ] && L=$K1
    bench_line $O v5_$v "$L" --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 --v5-ofuf || return 1
    bench_line $O v9_$v "$L" --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 || return 1
  done
}

tt16ab() {
  local O=gpurun_out/tt16ab; mkdir -p $O
  timeout -k 10 900 python -u -m pytest tests/test_gpu_tt.py tests/test_gpu_model.py -q -x --timeout 300 -k "tt or E3M4 or e3m4" \
    > $O/tests.log 2>&1 || { tail -5 $O/tests.log; return 1; }
  tail -1 $O/tests.log
  for v in ns2 ns1 f7ns1; do
    L=""; [ $v != ns2 ] && L=$AB/libfp8approx_$v.so
    bench_line $O r50_e3m4_$v "$L" --arch resnet50 --expo-width 3 --mant-width 4 --batch 512 || return 1
  done
}

splitab() {
  local O=gpurun_out/splitab; mkdir -p $O
  bench_line $O r18_def "" || return 1
  FP8A_SPLITK=1 bench_line $O r18_s1 "" || return 1
  bench_line $O r50_def "" --arch resnet50 --batch 512 || return 1
  FP8A_SPLITK=1 bench_line $O r50_s1 "" --arch resnet50 --batch 512 || return 1
}

bdma() {
  local O=gpurun_out/bdma; mkdir -p $O
  timeout -k 10 900 python -u -m pytest tests/test_gpu_f8mx.py tests/test_gpu_xm_shapes.py tests/test_gpu_f8_e5m2.py tests/test_gpu_chain.py \
    -q -x --timeout 300 > $O/tests.log 2>&1 || { tail -5 $O/tests.log; return 1; }
  tail -1 $O/tests.log
  for v in def w6all nobdma; do
    L=""; [ $v != def ] && L=$AB/libfp8approx_$v.so
    bench_line $O r18_$v "$L" || return 1
  done
  for v in def nobdma; do
    L=""; [ $v != def ] && L=$AB/libfp8approx_$v.so
    bench_line $O r50_$v "$L" --arch resnet50 --batch 512 || return 1
  done
}

dwops() {
  local O=gpurun_out/dwops; mkdir -p $O
  timeout -k 10 900 python -u -m pytest tests/test_gpu_tbx.py tests/test_gpu_chain.py tests/test_gpu_mbv2_layers.py \
    -q -x --timeout 300 > $O/tests.log 2>&1 || { tail -5 $O/tests.log; return 1; }
  tail -1 $O/tests.log
  for v in def r6base; do
    L=""; [ $v != def ] && L=$AB/libfp8approx_$v.so
    bench_line $O mbv2_e4m3_$v "$L" --arch mobilenet_v2 --batch 512 || return 1
    bench_line $O mbv2_e5m2_$v "$L" --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 || return 1
  done
}

tapt() {
  local O=gpurun_out/tapt; mkdir -p $O
  timeout -k 10 900 python -u -m pytest tests/test_gpu_tbx.py tests/test_gpu_chain.py tests/test_gpu_mbv2_layers.py \
    tests/test_gpu_model.py -q -x --timeout 300 > $O/tests.log 2>&1 || { tail -5 $O/tests.log; return 1; }
  tail -1 $O/tests.log
  for v in def tapt0; do
    L=""; [ $v != def ] && L=$AB/libfp8approx_$v.so
    bench_line $O mbv2_e4m3_$v "$L" --arch mobilenet_v2 --batch 512 || return 1
    bench_line $O mbv2_e5m2_$v "$L" --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 || return 1
  done
}

dwemit() {
  local O=gpurun_out/dwemit; mkdir -p $O
  timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_tbx.py tests/test_gpu_mbv2_layers.py \
    tests/test_gpu_model.py tests/test_gpu_graph.py -q -x --timeout 300 > $O/tests.log 2>&1 || { tail -5 $O/tests.log; return 1; }
  tail -1 $O/tests.log
  bench_line $O mbv2_e4m3 "" --arch mobilenet_v2 --batch 512 || return 1
  bench_line $O mbv2_e5m2 "" --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 || return 1
  for v in 0 1; do
    FP8A_MBV2_XCHAIN=$v bench_line $O mbv2_e4m3_x$v "" --arch mobilenet_v2 --batch 512 || return 1
    FP8A_MBV2_XCHAIN=$v bench_line $O mbv2_e5m2_x$v "" --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 || return 1
  done
}

multirank() { bash tools/dbg_multirank.sh; }

for e in "$@"; do $e || exit 1; done
