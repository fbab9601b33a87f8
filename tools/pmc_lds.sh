#!/bin/bash
# LDS / VALU utilisation counters of gemm_f8mx_kernel on one ResNet-18 layer, per library build.
# Usage: bash tools/pmc_lds.sh <layer> <variant>...   (variant: base or lib/<v>.so)
LAYER=$1; shift
R=$(pwd); L=$R/fp8_quantization_amd/lib
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = base ]; then f=$L/libfp8approx.so; else f=$L/$v.so; fi
  OUT=$R/gpurun_out/pmc_lds_$v; mkdir -p $OUT
  FP8A_LIB_PATH=$f timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --kernel-include-regex gemm_f8mx -f csv -d $OUT -o run -- \
    python $R/tools/gemm_bench.py --layers $LAYER --reps 3 > $OUT/log 2>&1 || exit 1
  python - "$OUT" "$v" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
g = m["GRBM_GUI_ACTIVE"]
print(sys.argv[2], " ".join(f"{k}={v:.4g}" for k, v in sorted(m.items())))
print(sys.argv[2], f"LDS_IDX_ACTIVE/(GRBM*256)={m['SQ_LDS_IDX_ACTIVE'] / (g * 256):.3f}",
      f"ACTIVE_INST_VALU/(GRBM*1024)={m['SQ_ACTIVE_INST_VALU'] / (g * 1024):.3f}",
      f"BUSY/GRBM={m['SQ_BUSY_CYCLES'] / g:.3f}")
PY
done
