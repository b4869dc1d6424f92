#!/bin/bash
# NF-level rates (tools/hook_bench.c) of the resident-kernel path against the
# launch path, 64 B and 1500 B frames, batches of 64 / 256 / 1024, depth 1 / 4:
#   tools/hook_resident.sh <tag>   -> gpurun_out/<tag>/hook_resident.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-hook_resident}
mkdir -p "$OUT"
B=$R/tools/build/hook_bench
for LEN in 64 1500; do
  for BATCH in 64 256 1024; do
    timeout -k 10 30 "$B" cpu $LEN $BATCH 2 >> "$OUT/hook_resident.jsonl" 2>> "$OUT/hook.err" || { echo "cpu failed"; exit 1; }
    for P in ZEROCOPY RESIDENT; do
      for D in 1 4; do
        timeout -k 10 30 "$B" async $LEN $BATCH 2 $P $D >> "$OUT/hook_resident.jsonl" 2>> "$OUT/hook.err" \
          || { echo "async $P $LEN $BATCH $D failed"; tail -5 "$OUT/hook.err"; exit 1; }
      done
    done
    timeout -k 10 30 "$B" sync $LEN $BATCH 2 RESIDENT >> "$OUT/hook_resident.jsonl" 2>> "$OUT/hook.err" \
      || { echo "sync RESIDENT $LEN $BATCH failed"; exit 1; }
  done
done
cat "$OUT/hook_resident.jsonl"
