set -o pipefail
O=gpurun_out/ttxk; mkdir -p $O
XK4=fp8_quantization_amd/lib/ab/libfp8approx_xk4.so
FP8A_LIB_PATH=$XK4 timeout -k 10 600 python -u -m pytest tests/test_gpu_tt.py -q -x --timeout 300 > $O/tests_xk4.log 2>&1; rc=$?; tail -1 $O/tests_xk4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/tt_band_layer.py > $O/layers_xk2.log 2>&1 || exit 1
FP8A_LIB_PATH=$XK4 timeout -k 10 400 python -u tools/tt_band_layer.py > $O/layers_xk4.log 2>&1 || exit 1
grep layer $O/layers_xk2.log; grep layer $O/layers_xk4.log
for v in xk2 xk4; do
  L=""; [ $v = xk4 ] && L=$XK4
  FP8A_LIB_PATH=$L timeout -k 10 400 python bench.py --arch resnet50 --expo-width 2 --mant-width 5 --batch 512 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', round(d['value'],1), d['roofline']['frac'])"
done
