set -o pipefail
TAG=${1:-r06i}
OUT=gpurun_out/$TAG; mkdir -p $OUT
XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_vs_reference.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_ab_build.log 2>&1 || { echo ab suite failed; tail -30 $OUT/gpu_tests_ab_build.log; exit 1; }
tail -1 $OUT/gpu_tests_ab_build.log
bash tools/gpu_check.sh $TAG
