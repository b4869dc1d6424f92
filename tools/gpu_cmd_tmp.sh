set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/lp_tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error" gpurun_out/lp_tests.log | head; exit 1; }
for r in 1 2 3; do
timeout -k 10 200 python tools/tune.py --workload 64 --rotate 13 --bpc 8 --rounds 5 --variants 1,5,2,0,1,0,32 >> gpurun_out/lp_tune.jsonl 2>>gpurun_out/lp_tune.err || { tail gpurun_out/lp_tune.err; exit 1; }
done
cut -c1-200 gpurun_out/lp_tune.jsonl
