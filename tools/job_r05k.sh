#!/bin/bash
# Round 5, step k: windowed 32-bit A path of the bf16 dense GEMM (stem conv) + dense kernel timing in
# the config-1 bench line: dense / fused-layer tests, config-1 evidence (trace, PMC, bench line).
set -o pipefail
OUT=gpurun_out/r05k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dense.py \
    tests/test_gpu_grouped_conv.py tests/test_gpu_mbv2_layers.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/job_evidence_r05.sh c1_mbv2_noapprox || exit 1
python -c "import json; d=json.load(open('gpurun_out/ev5/bench_r05_c1_mbv2_noapprox.json')); r=d['roofline']; print({k: r.get(k) for k in ('frac','kernel_frac','kernel_avg_ms','hbm_gbs','hbm_frac','valu_busy','traffic')})"
