#!/bin/bash
# Per-batch latency with W workers at once (tools/ctx_latency.c), RESIDENT
# (one shared resident kernel) vs ZEROCOPY launches:
#   tools/ctx_workers.sh <tag>  -> gpurun_out/<tag>/ctx_workers.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ctxw}
mkdir -p "$OUT"
for LEN in 64 1500; do
  for N in 64 256; do
    for W in 1 4 8 16; do
      for P in RESIDENT ZEROCOPY; do
        [ "$P" = ZEROCOPY ] && [ "$W" -gt 8 ] && continue
        for D in 1 4; do
          timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN $N 4000 $P $D $W >> "$OUT/ctx_workers.jsonl" 2>> "$OUT/ctx_workers.err" \
            || { echo "ctx $LEN $N $P $D $W failed"; tail -3 "$OUT/ctx_workers.err"; exit 1; }
        done
      done
    done
  done
done
cat "$OUT/ctx_workers.jsonl"
