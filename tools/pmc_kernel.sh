#!/bin/bash
# SQ / LDS counter passes (each its own run, kernel-trace only) over one kernel of a bench
# configuration, closed by tools/pmc_close.py.
# Usage: bash tools/pmc_kernel.sh <out tag> <kernel regex> <bench args...>
set -o pipefail
TAG=$1; K=$2; shift 2
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
B="$R/bench.py --no-cpu-baseline --no-graph --steps 2 --warmup 1 $*"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$K" -f csv -d $O/p$i -o run -- \
      python $B > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
cd $R && python tools/pmc_close.py $O/p1 $O/p2 > $O/close.txt && cat $O/close.txt
