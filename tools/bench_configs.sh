#!/bin/bash
# Bench lines of the other BASELINE configs (run from the repo root on the GPU box):
#   bash tools/bench_configs.sh <round-tag>  -> gpurun_out/bench_<tag>_<name>.json
set -o pipefail
T=${1:-r02}
run() { name=$1; shift; timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bench_${T}_$name.json 2> gpurun_out/bench_${T}_$name.err || exit 1; tail -1 gpurun_out/bench_${T}_$name.json | cut -c1-160; }
run resnet50 --arch resnet50
run mobilenet_v2 --arch mobilenet_v2
run vit_fc --arch vit_fc
run r50_e3m4 --arch resnet50 --expo-width 3 --mant-width 4
run r50_e2m5 --arch resnet50 --expo-width 2 --mant-width 5
run mbv2_e3m4 --arch mobilenet_v2 --expo-width 3 --mant-width 4
