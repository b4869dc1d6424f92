#!/bin/bash
# Header-sector placement probe (PROBE_PASS2) on the 1500 B footprint, and the
# attainable-read probe library against the summing kernel (bench 1500 / jumbo).
#   tools/probe_pass2.sh <tag>     (run ON the GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-probe_pass2}
mkdir -p "$OUT"
P=$R/tools/build/hbm_probe
cd "$R"
timeout -k 10 120 env PROBE_PASS2=1 $P 1048576 2048 256 1504 20 > "$OUT/pass2.jsonl" \
  && cat "$OUT/pass2.jsonl" \
  && for W in 1500 jumbo 64; do
       timeout -k 10 240 python bench.py --workload $W --secondary "" --cpu-seconds 0 > "$OUT/bench_$W.json" \
         2> "$OUT/bench_$W.err" || exit 1
       python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], r['step_us'], r.get('summing_kernel_alone'), r['attainable'])" "$OUT/bench_$W.json" $W
     done
