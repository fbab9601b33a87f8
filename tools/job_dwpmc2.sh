set -o pipefail
FP8A_LIB_PATH=$(pwd)/fp8_quantization_amd/lib/ab/libfp8approx_kyu1.so bash tools/pmc_kernel.sh dwpmc_tbsg_k1 conv_tbsg_kernel --arch mobilenet_v2 --batch 512 > /dev/null || exit 1
bash tools/pmc_kernel.sh dwpmc_tbsg_t conv_tbsg_kernel --arch mobilenet_v2 --batch 512 > /dev/null || exit 1
for d in dwpmc_tbsg_t dwpmc_tbsg_k1; do echo $d; head -1 gpurun_out/$d/close.txt | tr ' ' '\n' | grep -E "BANK|IDX|WAIT_ANY|WAVE_CYCLES|INSTS_VALU|GRBM"; grep -E "waves_per|valu_winstr|lds_array" gpurun_out/$d/close.txt; done
