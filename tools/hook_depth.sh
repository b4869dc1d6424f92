#!/bin/bash
# Two-phase hook: batches in flight per worker (1..3) at the reference's batch
# sizes (tools/hook_bench.c), run ON the GPU box:  tools/hook_depth.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-hook_depth}
mkdir -p "$OUT"
B=$R/tools/build/hook_bench
for LEN in 1500 64; do
  for BATCH in 64 256; do
    for D in 1 2 3; do
      timeout -k 10 30 "$B" async $LEN $BATCH 2 ZEROCOPY $D >> "$OUT/hook_depth.jsonl" 2>> "$OUT/hook_depth.err" \
        || { echo "hook_bench $LEN $BATCH $D failed"; tail -5 "$OUT/hook_depth.err"; exit 1; }
    done
    timeout -k 10 30 "$B" async $LEN $BATCH 2 STAGED 3 >> "$OUT/hook_depth.jsonl" 2>> "$OUT/hook_depth.err" \
      || { echo "hook_bench staged failed"; exit 1; }
  done
done
cat "$OUT/hook_depth.jsonl"
