set -o pipefail
OUT=gpurun_out/${1:-r06n}; mkdir -p $OUT
XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "pool_guard_trips or grid_sizing" -v --timeout 300 --timeout-method thread > $OUT/gpu_guard_ab.log 2>&1 || { echo tests failed; tail -40 $OUT/gpu_guard_ab.log; exit 1; }
tail -2 $OUT/gpu_guard_ab.log
