#!/bin/bash
# A/B (needs `make ab` and build/ab_clamp, the same with -DXSKNF_LANE_CLAMP=1):
# the lane kernel's chunk loads past the frame skipped (product) or clamped to
# its last chunk (round 3), shapes 5x2 (default), 5x1, 4x2, on 64 / 60 B
# frames, aligned and unaligned, worst case and NIC checks; libraries
# interleaved, 2 rounds each:
#   tools/ab_lane_pred.sh <tag>  -> gpurun_out/<tag>/ab_lane_pred.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ablp}
mkdir -p "$OUT"
for rep in 1 2; do
  for L in ab ab_clamp; do
    for W in 64 64u 60u; do
      for C in nic zero; do
        XSKNF_GPU_LIB=$R/build/$L/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/tune.py" --workload $W \
          --checks $C --rotate 13 --rounds 5 --variants "1,5,1,0,1:1,4,2,0,1" 2>> "$OUT/err" \
          | sed "s|^{|{\"lib\": \"$L\", \"rep\": $rep, |" >> "$OUT/ab_lane_pred.jsonl" || { tail -20 "$OUT/err"; exit 1; }
      done
    done
  done
done
python3 - "$OUT/ab_lane_pred.jsonl" <<'PY'
import json, sys, collections, statistics as st
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["checks"], tuple(j["shape"][:3]), j["lib"])].append(j["us"])
for k in sorted(d): print(k, d[k])
PY
