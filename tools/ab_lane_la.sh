#!/bin/bash
# A/B (round 5): the lane kernel's windows transposed per tile (XSKNF_LA(5, 2),
# window field 1024, the default since round 5) against per-lane loads (window
# 0), at a 1M-frame batch per launch and a 13M-frame batch in one launch, 64 B
# aligned worst case and NIC checks; 3 interleaved rounds in tune.py processes.
#   tools/ab_lane_la.sh <tag>   (ON the GPU box)  -> gpurun_out/<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ablla}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for FC in 1048576:13:zero 1048576:13:nic 13631488:1:zero; do
    IFS=: read F K C <<< "$FC"
    timeout -k 10 300 python "$R/tools/tune.py" --workload 64 --frames $F --rotate $K --checks $C --rounds 5 \
      --reps 5 --variants "1,5,2,0,1,0,0" 2>> "$OUT/err" | sed "s|^{|{\"rep\": $rep, \"frames\": $F, |" \
      >> "$OUT/ab.jsonl" || { tail -20 "$OUT/err"; exit 1; }
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["frames"], j["checks"], ",".join(map(str, j["shape"])))].append(j["us"])
for k in sorted(d): print(k, sorted(d[k]))
PY
