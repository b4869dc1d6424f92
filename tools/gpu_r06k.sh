set -o pipefail
OUT=gpurun_out/${1:-r06k}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_multi.py -k "packed or tool" -v --timeout 300 --timeout-method thread > $OUT/gpu_packed.log 2>&1 || { echo tests failed; tail -40 $OUT/gpu_packed.log; exit 1; }
tail -2 $OUT/gpu_packed.log
timeout -k 10 300 tools/build/multi_config4 > $OUT/multi_config4.json 2> $OUT/multi_config4.err || { echo tool failed; tail -20 $OUT/multi_config4.err; exit 1; }
cat $OUT/multi_config4.json
timeout -k 10 500 python -u tools/e2e_bench.py --paths zerocopy,staged,resident --orders rx,scattered --modes async --seconds 1.0 --check > $OUT/e2e.jsonl 2> $OUT/e2e.err || { echo e2e failed; tail -20 $OUT/e2e.err; exit 1; }
tail -3 $OUT/e2e.jsonl
