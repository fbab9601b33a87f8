set -o pipefail
O=gpurun_out/v5ab; mkdir -p $O
K1=fp8_quantization_amd/lib/ab/libfp8approx_v5k1.so
FP8A_LIB_PATH=$K1 timeout -k 10 600 python -u -m pytest tests/test_gpu_v5.py tests/test_gpu_chain.py -q -x --timeout 300 > $O/tests_k1.log 2>&1; rc=$?; tail -1 $O/tests_k1.log; [ $rc -eq 0 ] || exit $rc
run() {
  FP8A_LIB_PATH=$2 timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || { tail -3 $O/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1))"
}
run v5_base "" "--expo-width 5 --mant-width 2 --v5-ofuf"
run v5_k1 $K1 "--expo-width 5 --mant-width 2 --v5-ofuf"
run v9_base "" "--expo-width 5 --mant-width 2"
run v9_k1 $K1 "--expo-width 5 --mant-width 2"
run v5_base2 "" "--expo-width 5 --mant-width 2 --v5-ofuf"
run v5_k1b $K1 "--expo-width 5 --mant-width 2 --v5-ofuf"
