set -o pipefail
OUT=gpurun_out/${1:-r06o}; mkdir -p $OUT
XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "pool_guard_trips or grid_sizing or pool_units" -v --timeout 300 --timeout-method thread > $OUT/gpu_guard_ab.log 2>&1 || { echo ab tests failed; tail -40 $OUT/gpu_guard_ab.log; exit 1; }
tail -2 $OUT/gpu_guard_ab.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "grid_sizing or pool_units or full_size or every_launch_shape" -v --timeout 300 --timeout-method thread > $OUT/gpu_pool_product.log 2>&1 || { echo product tests failed; tail -40 $OUT/gpu_pool_product.log; exit 1; }
tail -2 $OUT/gpu_pool_product.log
bash tools/prof_all.sh r06o 1500 jumbo 1500-nic jumbo-nic || exit 1
