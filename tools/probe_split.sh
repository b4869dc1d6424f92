#!/bin/bash
# Write-side probes on the 1500 B footprint (1M chunks of 2048 B, frame at +256,
# 1504 B read): read modes, scatter shapes after a read pass, the side-buffer
# variant, and the K-sub-batch split (read + sector rewrite per sub-batch).
#   tools/probe_split.sh <tag>     (run ON the GPU box)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-probe_split}
mkdir -p "$OUT"
P=$R/tools/build/hbm_probe
timeout -k 10 120 env PROBE_MODES=1 PROBE_SEQ=1 PROBE_SIDE=1 $P 1048576 2048 256 1504 20 > "$OUT/modes_seq_side.jsonl" \
  && timeout -k 10 200 env PROBE_SPLIT=1 $P 1048576 2048 256 1504 12 > "$OUT/split.jsonl" \
  && cat "$OUT"/*.jsonl
