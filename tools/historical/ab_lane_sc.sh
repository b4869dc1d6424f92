#!/bin/bash
# A/B (round 5): the lane kernel's in-line sector stores nt (product) against
# write-through sc1 / sc0 sc1 / sc1 nt (build/lsc{1,2,3}: tools/build_variant.sh
# with -DXSKNF_LANE_SC=N), 64 B aligned worst case and NIC checks, 64 B packed;
# libraries interleaved, 2 rounds; then the per-wave timelines of nt and sc1.
#   tools/ab_lane_sc.sh <tag>  -> gpurun_out/<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ablsc}
mkdir -p "$OUT"
for rep in 1 2; do
  for L in lib lsc1 lsc2 lsc3; do
    LIB=$R/build/$L/libxsknf_gpu.so; [ $L = lib ] && LIB=$R/xsknf_amd/lib/libxsknf_gpu.so
    for WC in 64:zero 64:nic 64u:zero; do
      W=${WC%%:*}; C=${WC#*:}
      {
        XSKNF_GPU_LIB=$LIB timeout -k 10 200 python "$R/tools/tune.py" --workload $W \
          --checks $C --rotate 13 --rounds 5 2>> "$OUT/err" \
          | sed "s|^{|{\"lib\": \"$L\", \"rep\": $rep, |" >> "$OUT/ab_lane_sc.jsonl" || { tail -20 "$OUT/err"; exit 1; }
      }
    done
  done
done
for L in tl tl_lsc1; do
  XSKNF_GPU_LIB=$R/build/$L/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/timeline.py" --workload 64 \
    --rotate 13 --reps 20 2>> "$OUT/err" | sed "s|^{|{\"lib\": \"$L\", |" >> "$OUT/timeline_lane.jsonl" || { tail -20 "$OUT/err"; exit 1; }
done
python3 - "$OUT/ab_lane_sc.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["checks"], j["lib"])].append(j["us"])
for k in sorted(d): print(k, d[k])
PY
