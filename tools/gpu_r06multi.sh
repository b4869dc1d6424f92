set -o pipefail
OUT=gpurun_out/${1:-r06g}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -k "c_host" -x -v --timeout 300 --timeout-method thread -s > $OUT/gpu_multi.log 2>&1 || { echo tests failed; tail -40 $OUT/gpu_multi.log; exit 1; }
tail -3 $OUT/gpu_multi.log; grep "c-host" $OUT/gpu_multi.log
timeout -k 10 300 python bench.py --secondary "" --cpu-seconds 0 --no-probes > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'], json.dumps(d.get('c_host_multi')))"
wc -l $OUT/bench.json
