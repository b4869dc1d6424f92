set -o pipefail
OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 300 python -u tools/nf_start_probe.py --starts 40 --hold 0.3 --out $OUT/nf_start_probe.jsonl > $OUT/nf_start_probe.log 2>&1 || { echo probe failed; tail -20 $OUT/nf_start_probe.log; exit 1; }
tail -1 $OUT/nf_start_probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_app.py -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests failed; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log; grep "c-host multi" $OUT/gpu_tests.log
cp gpurun_out/nf_starts.jsonl $OUT/
timeout -k 10 300 python bench.py --secondary "" --cpu-seconds 0 --no-probes > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['roofline']['frac'], json.dumps(d.get('c_host_multi')))"
