#!/bin/bash
# NF-level rates for choosing checksummer_app's default host path per rx batch
# size (tools/hook_bench.c, the feeding thread pinned apart from the worker):
# the CPU NF, the launched hook (ZEROCOPY, 1 and 2 out) and the resident hook
# (4 out), 64 B and 1500 B frames, batches of 64 / 128 / 256 / 1024, REPS
# interleaved repetitions of 2 s each (the medians decide):
#   tools/hook_default.sh <tag> [REPS]   -> gpurun_out/<tag>/hook_default.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-hook_default}
REPS=${2:-5}
mkdir -p "$OUT"
B=$R/tools/build/hook_bench
for rep in $(seq 1 $REPS); do
  for LEN in 64 1500; do
    for BATCH in 64 128 256 1024; do
      for M in "cpu" "async ZEROCOPY 1" "async ZEROCOPY 2" "async RESIDENT 4"; do
        set -- $M
        line=$(timeout -k 10 30 "$B" $1 $LEN $BATCH 2 ${2:-ZEROCOPY} ${3:-1} 2>> "$OUT/hook.err") \
          || { echo "$M $LEN $BATCH failed"; tail -5 "$OUT/hook.err"; exit 1; }
        echo "{\"rep\": $rep, ${line#\{}" >> "$OUT/hook_default.jsonl"
      done
    done
  done
  echo "rep $rep done"
done
python3 - "$OUT/hook_default.jsonl" <<'PY'
import json, sys, statistics as st
rows = [json.loads(l) for l in open(sys.argv[1])]
key = lambda r: (r["len"], r["batch"], r["mode"] if r["mode"] == "cpu" else f'{r["path"]} d{r["depth"]}')
for k in sorted({key(r) for r in rows}):
    v = [r["mpps"] for r in rows if key(r) == k]
    print(k, "median %.2f" % st.median(v), "range %.2f-%.2f" % (min(v), max(v)))
PY
