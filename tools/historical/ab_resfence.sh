#!/bin/bash
# A/B (timing only): the resident kernel's system-scope fences vs none (build/resfence0)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-resfence}
mkdir -p "$OUT"
for rep in 1 2; do
  for V in default fence0; do
    for LEN in 64 1500; do
      for D in 1 4; do
        if [ $V = fence0 ]; then L="$R/build/resfence0"; else L=""; fi
        LD_LIBRARY_PATH=$L timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN 64 4000 RESIDENT $D \
          | sed "s/^{/{\"variant\": \"$V\", /" >> "$OUT/ctx.jsonl" || exit 1
      done
    done
  done
done
cat "$OUT/ctx.jsonl"
