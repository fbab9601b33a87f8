#!/bin/bash
# Round 5 evidence: per configuration a kernel trace + FETCH / WRITE / SQ PMC passes
# (tools/profile_config.sh), the PMC summary placed under profiles/ as pmc_r05_<tag>.json so the
# bench line that follows carries traffic / hbm_gbs / valu_busy / wave_cycles, the per-kernel
# breakdown and the rocprof summary.
# Usage: bash tools/job_evidence_r05.sh [tag ...]
set -o pipefail
OUT=gpurun_out/ev5; mkdir -p $OUT
declare -A SPEC=(
  [c1_mbv2_noapprox]="dn_gemm_bf16 mobilenet_v2 4 3 512 --no-approx"
  [c2_r18_e4m3]="gemm_f8mx_kernel resnet18 4 3 1024"
  [c3_mbv2_e5m2_v5]="gemm_v5mx_kernel mobilenet_v2 5 2 512 --v5-ofuf"
  [c3_mbv2_e5m2_v9]="gemm_f8mx_kernel mobilenet_v2 5 2 512"
  [c4_vit_b16]="gemm_f8mx_kernel vit_b16 4 3 64"
  [c5_r50_e4m3]="gemm_f8mx_kernel resnet50 4 3 512"
  [c5_r50_e5m2]="gemm_f8mx_kernel resnet50 5 2 512"
  [c5_r50_e3m4]="gemm_tt16_kernel resnet50 3 4 512"
  [c5_r50_e2m5]="gemm_tt_kernel resnet50 2 5 512"
  [mbv2_e4m3]="gemm_f8mx_kernel mobilenet_v2 4 3 512"
  [mbv2_e4m3_dw]="conv_tbs_kernel mobilenet_v2 4 3 512"
  [c1_mbv2_noapprox_dw]="dn_dw3g_kernel mobilenet_v2 4 3 512 --no-approx"
)
TAGS="$*"; [ -n "$TAGS" ] || TAGS="c2_r18_e4m3"
for t in $TAGS; do
  set -- ${SPEC[$t]}
  K=$1; ARCH=$2; E=$3; M=$4; B=$5; shift 5; EXTRA="$*"
  bash tools/profile_config.sh ev5_$t $K $ARCH $E $M $B $EXTRA > $OUT/$t.prof.log 2>&1 || { tail -5 $OUT/$t.prof.log; exit 1; }
  cp gpurun_out/ev5_$t/pmc.json $OUT/pmc_r05_$t.json && cp gpurun_out/ev5_$t/pmc.json profiles/pmc_r05_$t.json
  cp gpurun_out/ev5_$t/summary.txt $OUT/rocprof_r05_${t}_summary.txt
  python tools/trace_breakdown.py $(ls gpurun_out/ev5_$t/trace/*kernel_trace.csv) --forwards 5:3 \
      --out $OUT/breakdown_$t.txt > /dev/null || exit 1
  sed -n 2,8p $OUT/breakdown_$t.txt
  timeout -k 10 300 python bench.py --arch $ARCH --expo-width $E --mant-width $M --batch $B $EXTRA > $OUT/bench_r05_$t.json \
      2> $OUT/bench_r05_$t.err || { tail -3 $OUT/bench_r05_$t.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_r05_$t.json')); r=d.get('roofline') or {}; print('$t', round(d['value'],1), {k: r.get(k) for k in ('frac','op_frac','hbm_gbs','valu_busy')})"
done
