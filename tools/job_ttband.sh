set -o pipefail
bash tools/gpu_job.sh ttb "tests:test_gpu_tt or E2M5" || exit $?
FP8A_TT_BAND=0 bash tools/gpu_job.sh ttb bench:r50_e2m5_band0:--arch,resnet50,--expo-width,2,--mant-width,5,--batch,512,--no-cpu-baseline || exit $?
bash tools/gpu_job.sh ttb bench:r50_e2m5_band1:--arch,resnet50,--expo-width,2,--mant-width,5,--batch,512,--no-cpu-baseline || exit $?
