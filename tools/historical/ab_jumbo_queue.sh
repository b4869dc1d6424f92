#!/bin/bash
# A/B (round 5): jumbo's checks patched inside the launch from the pooled
# block's queue (build/jpt16: -DXSKNF_JUMBO_PT=16, shape fused_stores 2 + 16)
# against the product's per-tile policy + scatter_checks pass; worst case and
# NIC checks, 3 interleaved rounds; then the per-wave timeline of both.
#   tools/ab_jumbo_queue.sh <tag>  -> gpurun_out/<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-abjq}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for C in zero nic; do
    XSKNF_GPU_LIB=$R/xsknf_amd/lib/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/tune.py" --workload jumbo \
      --checks $C --rounds 5 2>> "$OUT/err" | sed "s|^{|{\"lib\": \"lib\", \"rep\": $rep, |" >> "$OUT/ab_jumbo.jsonl" \
      || { tail -20 "$OUT/err"; exit 1; }
    XSKNF_GPU_LIB=$R/build/jpt16/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/tune.py" --workload jumbo \
      --checks $C --rounds 5 --variants "16,3,2,0,18,1,52" 2>> "$OUT/err" \
      | sed "s|^{|{\"lib\": \"jpt16\", \"rep\": $rep, |" >> "$OUT/ab_jumbo.jsonl" || { tail -20 "$OUT/err"; exit 1; }
  done
done
XSKNF_GPU_LIB=$R/build/tl_jpt16/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/timeline.py" --workload jumbo \
  --reps 10 --variant "16,3,2,0,18,1,52" 2>> "$OUT/err" | sed "s|^{|{\"lib\": \"tl_jpt16\", |" >> "$OUT/timeline_jumbo.jsonl" \
  || { tail -20 "$OUT/err"; exit 1; }
XSKNF_GPU_LIB=$R/build/tl/libxsknf_gpu.so timeout -k 10 200 python "$R/tools/timeline.py" --workload jumbo \
  --reps 10 2>> "$OUT/err" | sed "s|^{|{\"lib\": \"tl\", |" >> "$OUT/timeline_jumbo.jsonl" || { tail -20 "$OUT/err"; exit 1; }
python3 - "$OUT/ab_jumbo.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["checks"], j["lib"], j["shape"][4], j["matches_default"])].append(j["us"])
for k in sorted(d): print(k, d[k])
PY
