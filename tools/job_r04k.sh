#!/bin/bash
# Round 4: block-size sweep of the LDS-staged depthwise kernels (options dw_target / dw_lds) on the
# MobileNetV2 bench lines, and SQ counters of dn_dw3_kernel / conv_tbs_kernel.
set -o pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grouped_conv.py \
    tests/test_gpu_tbx.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for tl in 1024:20480 2048:20480 4096:40960 8192:65536; do
  t=${tl%%:*}; l=${tl#*:}
  for spec in "c1:--arch mobilenet_v2 --no-approx" "mb:--arch mobilenet_v2"; do
    tag=${spec%%:*}; a=${spec#*:}
    FP8A_DW_TARGET=$t FP8A_DW_LDS=$l timeout -k 10 300 python bench.py $a --no-cpu-baseline --steps 10 > $OUT/bench_${tag}_$t.json 2> $OUT/bench_${tag}_$t.err || exit $?
    echo "$tag target $t lds $l $(python -c "import json,sys; print(round(json.load(open('$OUT/bench_${tag}_$t.json'))['value']))")"
  done
done
cd /tmp && export TMPDIR=/tmp
for spec in "c1:dn_dw3:--arch mobilenet_v2 --no-approx" "mb:conv_tbs:--arch mobilenet_v2"; do
  tag=${spec%%:*}; rest=${spec#*:}; kre=${rest%%:*}; a=${rest#*:}
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex $kre -f csv -d $R/$OUT/pmc_${tag}_1 -o run -- \
    python $R/bench.py $a --no-cpu-baseline --steps 2 --warmup 1 > $R/$OUT/pmc_${tag}_1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
    SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-include-regex $kre -f csv -d $R/$OUT/pmc_${tag}_2 -o run -- \
    python $R/bench.py $a --no-cpu-baseline --steps 2 --warmup 1 > $R/$OUT/pmc_${tag}_2.log 2>&1 || exit $?
  python - $R/$OUT/pmc_$tag <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "_*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
print(sys.argv[1].split("/")[-1], " ".join(f"{k}={v:.4g}" for k, v in sorted(m.items())))
wc = m.get("SQ_WAVE_CYCLES", 0) or 1
print("  wait_any/wave_cycles %.3f  wait_inst_any %.3f  active_inst_any %.3f  valu busy/(GRBM*1024) %.3f" % (
    m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
    m.get("SQ_ACTIVE_INST_VALU", 0) / (m.get("GRBM_GUI_ACTIVE", 1) * 1024)))
PY
done
