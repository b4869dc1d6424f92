#!/bin/bash
# A/B: resident ring geometry (entries x frames per entry): the product's 8 x 256
# against build/res16x64 and build/res16x128 (XSKNF_RES_SLOTS / _FRAMES), per-batch
# latency (ctx_latency) and NF level (hook_bench), interleaved in one process tree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-resring}
mkdir -p "$OUT"
for rep in 1 2; do
  for V in default 16x64 16x128; do
    if [ $V = default ]; then L=""; else L="$R/build/res$V"; fi
    for LEN in 64 1500; do
      for N in 64 256; do
        for D in 1 4; do
          LD_LIBRARY_PATH=$L timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN $N 4000 RESIDENT $D \
            | sed "s/^{/{\"ring\": \"$V\", /" >> "$OUT/ctx.jsonl" || exit 1
        done
        LD_LIBRARY_PATH=$L timeout -k 5 30 "$R/tools/build/hook_bench" async $LEN $N 2 RESIDENT 4 \
          | sed "s/^{/{\"ring\": \"$V\", /" >> "$OUT/hook.jsonl" || exit 1
      done
    done
  done
done
cat "$OUT/ctx.jsonl" "$OUT/hook.jsonl"
