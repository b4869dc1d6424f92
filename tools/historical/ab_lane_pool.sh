#!/bin/bash
# A/B (round 5): the lane kernel (64 B) with the CU-wide tile pool in 64-frame
# units (one 16-wave block per CU) against the static 4-wave blocks; builds
# lpool (-DXSKNF_LANE_POOL_AB) and lpool_sc3 (+ sc1 nt sector stores); 64 B
# aligned worst case and NIC checks, 64 B packed; 2 interleaved rounds; then
# the per-wave timeline of the pooled shape.
#   tools/ab_lane_pool.sh <tag>  -> gpurun_out/<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ablp}
mkdir -p "$OUT"
for rep in 1 2; do
  for L in lpool lpool_sc3; do
    for WC in 64:zero 64:nic 64u:zero; do
      W=${WC%%:*}; C=${WC#*:}
      XSKNF_GPU_LIB=$R/build/$L/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/tune.py" --workload $W \
        --checks $C --rotate 13 --rounds 5 --variants "1,5,1,0,1,0,32:1,5,2,0,1,0,32" 2>> "$OUT/err" \
        | sed "s|^{|{\"lib\": \"$L\", \"rep\": $rep, |" >> "$OUT/ab_lane_pool.jsonl" || { tail -20 "$OUT/err"; exit 1; }
    done
  done
done
XSKNF_GPU_LIB=$R/build/tl_lpool/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/timeline.py" --workload 64 \
  --rotate 13 --reps 20 --variant "1,5,1,0,1,0,32" 2>> "$OUT/err" | sed "s|^{|{\"lib\": \"tl_lpool\", |" \
  >> "$OUT/timeline_lane_pool.jsonl" || { tail -20 "$OUT/err"; exit 1; }
python3 - "$OUT/ab_lane_pool.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["checks"], j["lib"], tuple(j["shape"][1:3]), j["shape"][6], j["matches_default"])].append(j["us"])
for k in sorted(d): print(k, d[k])
PY
