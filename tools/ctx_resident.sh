#!/bin/bash
# Per-batch latency of the host paths (tools/ctx_latency.c), launched vs resident:
#   tools/ctx_resident.sh <tag>  -> gpurun_out/<tag>/ctx.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ctx}
mkdir -p "$OUT"
for LEN in 64 1500; do
  for N in 64 256; do
    for P in ZEROCOPY RESIDENT; do
      for D in 1 4; do
        timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN $N 4000 $P $D >> "$OUT/ctx.jsonl" 2>> "$OUT/ctx.err" \
          || { echo "ctx $LEN $N $P $D failed"; tail -3 "$OUT/ctx.err"; exit 1; }
      done
    done
  done
done
cat "$OUT/ctx.jsonl"
