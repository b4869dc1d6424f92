#!/bin/bash
# A/B: blocks per resident ring entry (XSKNF_RES_GROUP): the product's group
# against build/resg1 (one block per entry, the previous geometry), per-batch
# latency (ctx_latency) at 64 / 256 / 1024 frames and NF level (hook_bench),
# interleaved.  Hypothesis: a 256-frame batch dealt over 4 blocks (one round of
# PCIe reads each) cuts its round trip >= 30 % without costing 64-frame batches
# more than 5 %.
#   make all tools && hipcc ... -DXSKNF_RES_GROUP=1 -o build/resg1/libxsknf_gpu.so
#   tools/ab_resgroup.sh <tag>  -> gpurun_out/<tag>/{ctx,hook}.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-resgroup}
mkdir -p "$OUT"
for rep in 1 2; do
  for V in default g1; do
    if [ $V = default ]; then L=""; else L="$R/build/res$V"; fi
    for LEN in 64 1500; do
      for N in 64 256 1024; do
        for D in 1 4; do
          LD_LIBRARY_PATH=$L timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN $N 4000 RESIDENT $D \
            | sed "s/^{/{\"group\": \"$V\", /" >> "$OUT/ctx.jsonl" || exit 1
        done
        LD_LIBRARY_PATH=$L timeout -k 5 30 "$R/tools/build/hook_bench" async $LEN $N 2 RESIDENT 4 \
          | sed "s/^{/{\"group\": \"$V\", /" >> "$OUT/hook.jsonl" || exit 1
      done
    done
  done
done
cat "$OUT/ctx.jsonl" "$OUT/hook.jsonl"
