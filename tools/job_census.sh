set -o pipefail
bash tools/gpu_job.sh g7 "tests:multirank or graph" bench:default || exit $?
mkdir -p gpurun_out/census
for cfg in "resnet50 2 5" "resnet50 3 4" "resnet18 4 3" "mobilenet_v2 4 3"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/census.py --arch $1 --expo-width $2 --mant-width $3 --batch 16 --tiles \
     --out gpurun_out/census/census_$1_e$2m$3.json > gpurun_out/census/census_$1_e$2m$3.txt 2>&1 || { tail -5 gpurun_out/census/census_$1_e$2m$3.txt; exit 1; }
  head -1 gpurun_out/census/census_$1_e$2m$3.txt
done
