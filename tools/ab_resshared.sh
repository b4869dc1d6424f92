#!/bin/bash
# A/B: the shared resident kernel (product lib) vs the per-context one of
# round 3 (build/old), one worker, interleaved, 3 rounds:
#   tools/ab_resshared.sh <tag>  -> gpurun_out/<tag>/ab.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-abres}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for LEN in 64 1500; do
    for N in 64 256; do
      for D in 1 4; do
        for V in new old; do
          if [ $V = old ]; then LIBP=$R/build/old; else LIBP=$R/xsknf_amd/lib; fi
          line=$(LD_LIBRARY_PATH=$LIBP timeout -k 5 60 "$R/tools/build/ctx_latency" $LEN $N 4000 RESIDENT $D 2>> "$OUT/ab.err") \
            || { echo "ab $V $LEN $N $D failed"; tail -3 "$OUT/ab.err"; exit 1; }
          echo "{\"variant\": \"$V\", \"rep\": $rep, ${line#\{}" >> "$OUT/ab.jsonl"
        done
      done
    done
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, statistics as st
rows = [json.loads(l) for l in open(sys.argv[1])]
keys = sorted({(r["len"], r["n"], r["depth"]) for r in rows})
for k in keys:
    m = {v: st.median(r["us_per_batch"] for r in rows if (r["len"], r["n"], r["depth"]) == k and r["variant"] == v)
         for v in ("new", "old")}
    print(k, m)
PY
