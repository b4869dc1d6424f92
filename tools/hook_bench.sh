#!/bin/bash
# NF-level rates of the worker loop (tools/hook_bench.c) on the GPU box:
#   tools/hook_bench.sh <tag>   -> gpurun_out/<tag>/hook_bench.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-hook_bench}
mkdir -p "$OUT"
B=$R/tools/build/hook_bench
for LEN in 64 1500; do
  for BATCH in 64 256 1024; do
    for MODE in null cpu sync async; do
      timeout -k 10 30 "$B" $MODE $LEN $BATCH 2 >> "$OUT/hook_bench.jsonl" 2>> "$OUT/hook_bench.err" \
        || { echo "hook_bench $MODE $LEN $BATCH failed"; tail -5 "$OUT/hook_bench.err"; exit 1; }
    done
    timeout -k 10 30 "$B" async $LEN $BATCH 2 STAGED >> "$OUT/hook_bench.jsonl" 2>> "$OUT/hook_bench.err" \
      || { echo "hook_bench staged $LEN $BATCH failed"; exit 1; }
  done
done
cat "$OUT/hook_bench.jsonl"
