#!/bin/bash
# Round 4: second block-plan sweep of the staged depthwise kernels (dw_target / dw_lds) after the
# aligned-slot staging; MobileNetV2 config 1 and E4M3 bench lines.
set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
for tl in 4096:40960 4096:32768 4096:49152 4096:65536 6144:49152 3072:32768; do
  t=${tl%%:*}; l=${tl#*:}
  for spec in "c1:--arch mobilenet_v2 --no-approx" "mb:--arch mobilenet_v2"; do
    tag=${spec%%:*}; a=${spec#*:}
    FP8A_DW_TARGET=$t FP8A_DW_LDS=$l timeout -k 10 300 python bench.py $a --no-cpu-baseline --steps 10 > $OUT/bench_${tag}_${t}_$l.json 2> $OUT/bench_${tag}_${t}_$l.err || exit $?
    echo "$tag target $t lds $l $(python -c "import json; print(round(json.load(open('$OUT/bench_${tag}_${t}_$l.json'))['value']))")"
  done
done
