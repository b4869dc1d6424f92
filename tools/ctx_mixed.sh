#!/bin/bash
# A mixed set of workers on one device (tools/ctx_latency.c with a path list):
# W RESIDENT workers alone, W ZEROCOPY workers alone, and W of each at once in
# one process, so the resident kernel's hardware queue sits beside the
# launches' streams (GPU_MAX_HW_QUEUES 4); 64-frame and 256-frame batches of
# 64 B, four batches out; 3 repetitions:
#   tools/ctx_mixed.sh <tag>  -> gpurun_out/<tag>/ctx_mixed.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ctxm}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for N in 64 256; do
    for W in 2 4; do
      for P in RESIDENT ZEROCOPY RESIDENT,ZEROCOPY; do
        NW=$W; [ "$P" = RESIDENT,ZEROCOPY ] && NW=$((2 * W))
        timeout -k 5 60 "$R/tools/build/ctx_latency" 64 $N 4000 $P 4 $NW | sed "s|^{|{\"rep\": $rep, |" \
          >> "$OUT/ctx_mixed.jsonl" 2>> "$OUT/ctx_mixed.err" || { echo "ctx $N $P $NW failed"; tail -3 "$OUT/ctx_mixed.err"; exit 1; }
      done
    done
  done
done
cat "$OUT/ctx_mixed.jsonl"
