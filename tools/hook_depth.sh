#!/bin/bash
# NF-level rates (tools/hook_bench.c) of the resident ring against batches out
# (depth 4 / 6 / 8), beside the CPU NF and the launched hook, 64 B and 1500 B
# frames, batches of 64 and 256:
#   tools/hook_depth.sh <tag>   -> gpurun_out/<tag>/hook_depth.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-hook_depth}
mkdir -p "$OUT"
B=$R/tools/build/hook_bench
for LEN in 64 1500; do
  for BATCH in 64 256; do
    timeout -k 10 30 "$B" cpu $LEN $BATCH 2 >> "$OUT/hook_depth.jsonl" 2>> "$OUT/hook.err" || { echo "cpu failed"; exit 1; }
    timeout -k 10 30 "$B" async $LEN $BATCH 2 ZEROCOPY 2 >> "$OUT/hook_depth.jsonl" 2>> "$OUT/hook.err" \
      || { echo "async ZEROCOPY $LEN $BATCH failed"; tail -5 "$OUT/hook.err"; exit 1; }
    for D in 4 6 8; do
      timeout -k 10 30 "$B" async $LEN $BATCH 2 RESIDENT $D >> "$OUT/hook_depth.jsonl" 2>> "$OUT/hook.err" \
        || { echo "async RESIDENT $LEN $BATCH $D failed"; tail -5 "$OUT/hook.err"; exit 1; }
    done
  done
done
cat "$OUT/hook_depth.jsonl"
