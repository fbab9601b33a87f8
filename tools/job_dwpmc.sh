set -o pipefail
bash tools/pmc_kernel.sh dwpmc_tbsg conv_tbsg_kernel --arch mobilenet_v2 --batch 512 || exit 1
bash tools/pmc_kernel.sh dwpmc_v5ds conv_v5ds_kernel --arch mobilenet_v2 --batch 512 --expo-width 5 --mant-width 2 --v5-ofuf || exit 1
bash tools/gpu_job.sh ev6 evidence:mbv2_e4m3_dw || exit 1
