#!/bin/bash
# Round 5, step a: where gemm_f8mx_kernel's issue slots go.
# 1. tools/seg_bench: products per SIMD-cycle of the kernel's instruction stream by parts;
# 2. SQ counters of the ResNet-18 l3.c2 dispatch (tools/gemm_bench.py), three PMC passes whose
#    WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY should close against SQ_WAVE_CYCLES.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/${1:-r05a}; mkdir -p $OUT
timeout -k 10 120 tools/bin/seg_bench 400 > $OUT/seg_bench.txt 2>&1 || exit $?
cat $OUT/seg_bench.txt
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex gemm_f8mx -f csv -d $OUT/pmc$i -o run -- \
    python $R/tools/gemm_bench.py --layers l3.c2 --reps 3 > $OUT/pmc$i.log 2>&1 || exit $?
done
python $R/tools/pmc_close.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 | tee $OUT/pmc_close.txt
