set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pool_tests.log 2>&1; rc=$?; tail -3 gpurun_out/pool_tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error" gpurun_out/pool_tests.log | head; exit 1; }
VARIANTS=16,2,2,0,18,1,56 bash tools/ab_dyn.sh pool1 xsknf_amd/lib || exit 1
bash tools/timeline.sh tl7 1500:16,2,2,0,18,1,56 570:16,2,2,0,18,1,56 imix:16,2,2,0,18,1,56
