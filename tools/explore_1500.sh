#!/bin/bash
# 1500 B exploration (run ON the GPU box): the attainable-read probe's shapes one
# by one, and the summing kernel's launch shapes in records-only mode (A/B build).
#   tools/explore_1500.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-explore_1500}
mkdir -p "$OUT"
cd "$R"
[ -n "$SKIP_PROBE" ] || timeout -k 10 240 env HBM_PROBE_VERBOSE=1 python bench.py --secondary "" --cpu-seconds 0 > "$OUT/bench.json" \
    2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
[ -n "$SKIP_PROBE" ] || grep hbm_probe "$OUT/bench.err"
timeout -k 10 400 env XSKNF_GPU_LIB=$R/build/ab/libxsknf_gpu.so python tools/tune.py --workload 1500 \
    --variants "16,3,1,0,3,1,24:16,3,2,0,3,1,24:16,2,2,0,3,1,24:16,4,1,0,3,1,24:32,3,1,0,3,1,24:16,2,1,0,3,1,24" \
    --bpc 4,8 > "$OUT/tune.jsonl" 2> "$OUT/tune.err" || { tail "$OUT/tune.err"; exit 1; }
cat "$OUT/tune.jsonl"
