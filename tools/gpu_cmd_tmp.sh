set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/j_tests.log 2>&1; rc=$?; tail -3 gpurun_out/j_tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error" gpurun_out/j_tests.log | head; exit 1; }
XSKNF_GPU_LIB=$PWD/build/ab/libxsknf_gpu.so timeout -k 10 300 python tools/tune.py --workload jumbo --bpc 4 --rounds 3 --reps 4 --variants 16,3,2,0,0,1,52:16,3,2,0,0,1,116:16,3,2,0,18,1,52 > gpurun_out/j_tune.jsonl 2>gpurun_out/j_tune.err || { tail gpurun_out/j_tune.err; exit 1; }
cut -c1-200 gpurun_out/j_tune.jsonl
