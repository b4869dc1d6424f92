#!/bin/bash
# Whole-step A/B of split-kernel shapes (A/B build, run ON the GPU box).
#   tools/explore_step.sh <tag> <workload> <variants>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-explore_step}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 env XSKNF_GPU_LIB=$R/build/ab/libxsknf_gpu.so python tools/tune.py --workload $2 \
    --variants "$3" --bpc ${BPC:-4,8} > "$OUT/tune_$2.jsonl" 2> "$OUT/tune_$2.err" || { tail "$OUT/tune_$2.err"; exit 1; }
cat "$OUT/tune_$2.jsonl"
