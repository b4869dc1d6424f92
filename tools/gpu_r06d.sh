set -o pipefail
bash tools/gpu_check.sh "${1:-r06e}" --starts "${2:-20}"
