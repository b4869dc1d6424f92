set -o pipefail
OUT=gpurun_out/${1:-r06j}; mkdir -p $OUT
XSKNF_GPU_CU_LIMIT=8 timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
  -k "not resident_contexts_share_one_kernel and not resident_rings_past_the_device_limit" > $OUT/gpu_tests_cu8.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests_cu8.log; grep -E "FAILED|ERROR" $OUT/gpu_tests_cu8.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "cu8 suite rc=$rc"; exit 1; }
timeout -k 10 300 python bench.py --secondary "" --cpu-seconds 0 --no-probes > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'], json.dumps(d['c_host_multi']['packed_round_trip']))"
