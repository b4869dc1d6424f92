#!/bin/bash
# A/B (round 5): IMIX with the checks of frames <= 128 B
# written in-line in phase A as their whole sector from the window (build/d129:
# -DXSKNF_DEFER2_MIN=129 -DXSKNF_DEFER_TILE_K=0), only longer frames' checks
# deferred to the patch list; against the product (every check deferred).
# Stop rule: adopt at >= 3 us on IMIX with 570 B and 1500 B not slower.
#   tools/ab_imix_inline.sh <tag>  -> gpurun_out/<tag>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-abii}
mkdir -p "$OUT"
for rep in 1 2 3; do
  for L in lib d129; do
    LIB=$R/build/$L/libxsknf_gpu.so; [ $L = lib ] && LIB=$R/xsknf_amd/lib/libxsknf_gpu.so
    for WC in imix:zero:4 imix:nic:4 570:zero:2 1500:zero:1; do
      IFS=: read W C K <<< "$WC"
      XSKNF_GPU_LIB=$LIB timeout -k 10 200 python "$R/tools/tune.py" --workload $W --checks $C --rotate $K \
        --rounds 5 2>> "$OUT/err" | sed "s|^{|{\"lib\": \"$L\", \"rep\": $rep, |" >> "$OUT/ab_imix_inline.jsonl" \
        || { tail -20 "$OUT/err"; exit 1; }
    done
  done
done
python3 - "$OUT/ab_imix_inline.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["checks"], j["lib"])].append(j["us"])
for k in sorted(d): print(k, d[k])
PY
