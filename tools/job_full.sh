set -o pipefail
bash tools/gpu_job.sh full tests smoke bench:default
