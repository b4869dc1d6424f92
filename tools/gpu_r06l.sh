set -o pipefail
OUT=gpurun_out/${1:-r06l}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -k "c_host or packed or tool" -v --timeout 300 --timeout-method thread > $OUT/gpu_multi.log 2>&1 || { echo tests failed; tail -40 $OUT/gpu_multi.log; exit 1; }
tail -2 $OUT/gpu_multi.log
