set -o pipefail
O=gpurun_out/dwab; mkdir -p $O
K1=fp8_quantization_amd/lib/ab/libfp8approx_kyu1.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_tbx.py tests/test_gpu_chain.py -q -x --timeout 300 > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
FP8A_LIB_PATH=$K1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tbx.py -q -x --timeout 300 > $O/tests_k1.log 2>&1; rc=$?; tail -1 $O/tests_k1.log; [ $rc -eq 0 ] || exit $rc
run() {  # name lib target lds
  FP8A_LIB_PATH=$2 FP8A_DW_TARGET=$3 FP8A_DW_LDS=$4 timeout -k 10 300 python bench.py --arch mobilenet_v2 --batch 512 --no-cpu-baseline > $O/$1.json 2> $O/$1.err || { tail -3 $O/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value'],1), round(d['hip_graph']['eager_images_per_s'],1))"
}
run base "" 4096 40960
run k1_4096 $K1 4096 40960
run k1_2048 $K1 2048 20480
run k1_1024 $K1 1024 12288
run base2 "" 4096 40960
run k1_2048b $K1 2048 20480
