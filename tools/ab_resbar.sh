#!/bin/bash
# A/B: the resident ring's headers and descriptors in device memory written
# through the BAR (default on large-BAR devices) vs in host memory (XSKNF_RESIDENT_BAR=0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-resbar}
mkdir -p "$OUT"
for rep in 1 2; do
  for BAR in 1 0; do
    for LEN in 64 1500; do
      for N in 64 256; do
        for D in 1 4; do
          XSKNF_RESIDENT_BAR=$BAR timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN $N 4000 RESIDENT $D \
            | sed "s/^{/{\"bar\": $BAR, /" >> "$OUT/ctx.jsonl" || exit 1
        done
      done
    done
  done
done
cat "$OUT/ctx.jsonl"
