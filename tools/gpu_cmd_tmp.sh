set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mid_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mid_tests.log
[ $rc = 0 ] || { grep -E "FAILED|Error" gpurun_out/mid_tests.log | head; exit 1; }
VARIANTS=16,2,2,0,18,1,24 bash tools/ab_dyn.sh mid1 xsknf_amd/lib build/d1 || exit 1
bash tools/timeline.sh tl11 1500 570 imix
