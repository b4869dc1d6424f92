set -o pipefail
OUT=gpurun_out/${1:-r06s}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_multi.py -k "packed or tool" -v --timeout 300 --timeout-method thread > $OUT/gpu_packed.log 2>&1 || { echo tests failed; tail -40 $OUT/gpu_packed.log; exit 1; }
tail -1 $OUT/gpu_packed.log
bash tools/gpu_r06r.sh ${1:-r06s}_prof
