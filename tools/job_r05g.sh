#!/bin/bash
# Round 5, step g: the depthwise layer set (tools/dw_bench.py) over staging form and block plan,
# and SQ / TA counters of the two staged forms on the first (largest) layer.
set -o pipefail
OUT=gpurun_out/r05g; mkdir -p $OUT
R=$(pwd)
for cfg in "1 4096 40960" "2 4096 40960" "2 2048 40960" "2 8192 65536" "2 16384 65536" "1 8192 65536" "2 1024 16384"; do
  set -- $cfg
  timeout -k 10 300 python tools/dw_bench.py --dw3 $1 --target $2 --lds $3 --qin > $OUT/dw_$1_$2_$3.log 2>&1 || { tail -5 $OUT/dw_$1_$2_$3.log; exit 1; }
  echo "$cfg $(tail -1 $OUT/dw_$1_$2_$3.log)"
done
head -3 $OUT/dw_1_4096_40960.log
head -3 $OUT/dw_2_4096_40960.log
for dw in 1 2; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
     SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex dn_dw3 -f csv -d $R/$OUT/pmc_dw$dw -o run -- \
     python $R/tools/dw_bench.py --dw3 $dw --qin --reps 1 > $R/$OUT/pmc_dw$dw.log 2>&1) || exit 1
done
echo done
