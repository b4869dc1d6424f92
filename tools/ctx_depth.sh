#!/bin/bash
# Per-batch time of the resident ring against batches out (tools/ctx_latency.c,
# depth 1..8; the ring has 8 entries), 64 frames of 64 B / 1500 B:
#   tools/ctx_depth.sh <tag>  -> gpurun_out/<tag>/ctx_depth.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ctx_depth}
mkdir -p "$OUT"
for LEN in 64 1500; do
  for P in ZEROCOPY RESIDENT; do
    for D in 1 2 4 6 8; do
      timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN 64 20000 $P $D >> "$OUT/ctx_depth.jsonl" 2>> "$OUT/ctx.err" \
        || { echo "ctx $LEN $P $D failed"; tail -3 "$OUT/ctx.err"; exit 1; }
    done
  done
done
cat "$OUT/ctx_depth.jsonl"
