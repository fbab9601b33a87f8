#!/bin/bash
# Round 5: bench.py's capture in thread_local error mode -- the default line and config 1.
set -o pipefail
OUT=gpurun_out/r05gr; mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/default.json 2> $OUT/default.err || { tail -5 $OUT/default.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/default.json')); print('default', round(d['value'],1), d['hip_graph'].get('captured'), d['hip_graph'].get('replay_matches_eager_bitwise'))"
timeout -k 10 300 python bench.py --arch mobilenet_v2 --no-approx --no-cpu-baseline > $OUT/c1.json 2> $OUT/c1.err || { tail -5 $OUT/c1.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c1.json')); print('c1', round(d['value'],1), d['hip_graph'].get('captured'))"
