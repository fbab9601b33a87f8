#!/bin/bash
# MobileNetV2 E4M3 with the round-3 defaults: bench line, profile_config evidence (trace + FETCH /
# WRITE), and SQ counter passes over the two depthwise kernels (conv_tbx_kernel default,
# conv_dwx_kernel opt-in) for the DESIGN comparison.
set -o pipefail
OUT=gpurun_out/mbpmc; mkdir -p $OUT
timeout -k 10 300 python bench.py --arch mobilenet_v2 --steps 5 --warmup 2 > $OUT/mb.json 2> $OUT/mb.err || exit $?
cat $OUT/mb.json | cut -c1-300
bash tools/profile_config.sh mb_e4m3_r3 gemm_f8mx_kernel mobilenet_v2 4 3 512 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
python tools/trace_breakdown.py $(ls gpurun_out/mb_e4m3_r3/trace/*kernel_trace.csv) --forwards 5:3 --out gpurun_out/mb_e4m3_r3/breakdown.txt | sed -n 2,14p
R=$(pwd); cd /tmp && export TMPDIR=/tmp
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $CTR --kernel-include-regex conv_tbx_kernel -f csv -d $R/$OUT/pmc_tbx -o run -- python $R/bench.py --arch mobilenet_v2 --steps 1 --warmup 0 --no-cpu-baseline > $R/$OUT/pmc_tbx.log 2>&1 || exit $?
FP8A_DWX=1 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $CTR --kernel-include-regex conv_dwx_kernel -f csv -d $R/$OUT/pmc_dwx -o run -- python $R/bench.py --arch mobilenet_v2 --steps 1 --warmup 0 --no-cpu-baseline > $R/$OUT/pmc_dwx.log 2>&1 || exit $?
cd $R && python - <<'PY'
import csv, collections, glob
for k in ("tbx", "dwx"):
    f = glob.glob(f"gpurun_out/mbpmc/pmc_{k}/*counter_collection.csv")[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.defaultdict(float)
    for d in per.values():
        for c, v in d.items(): tot[c] += v
    wc = tot["SQ_WAVE_CYCLES"] or 1
    print(k, {c: round(v / wc, 3) for c, v in tot.items() if c != "SQ_WAVE_CYCLES"}, "waves", tot["SQ_WAVES"], "instr/wave", round(tot["SQ_INSTS_VALU"] / max(1, tot["SQ_WAVES"]), 1))
PY
