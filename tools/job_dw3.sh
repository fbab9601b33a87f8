#!/bin/bash
set -o pipefail
bash tools/job_dwg_ab.sh || exit $?
R=$(pwd); cd /tmp && export TMPDIR=/tmp
FP8A_DW=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/dw3/trace -o run -- python $R/bench.py --arch mobilenet_v2 --steps 3 --warmup 1 --no-cpu-baseline > /tmp/dw3trace.log 2>&1 || exit $?
cd $R && python tools/trace_breakdown.py $(ls gpurun_out/dw3/trace/*kernel_trace.csv) --forwards 5:3 --out gpurun_out/dw3/breakdown.txt | sed -n 2,12p
