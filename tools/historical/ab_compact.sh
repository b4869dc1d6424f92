#!/bin/bash
# A/B (needs `make ab`): the compact split shape -- W = 8, 16 x 2, one item in
# flight, phase B's scratch in the window slots, a 4-tile patch list: 114 VGPRs
# and 40 KiB per 4-wave block, so 4 waves per SIMD -- against the IMIX default
# (the same with two items in flight: 160 VGPRs, 51 KiB, 3 waves per SIMD) and
# the pooled 12-wave shape, on IMIX (worst case and NIC checks), 570 B and
# 1500 B; one process per workload, shapes interleaved (tools/tune.py):
#   tools/ab_compact.sh <tag>  -> gpurun_out/<tag>/ab_compact.jsonl
# ABC_LIB (default build/ab) and ABC_VARIANTS override the library and shapes:
# build/ab_big (the A/B build with -DXSKNF_BIG_STATIC=1: blocks of more than 4
# waves deal their tiles statically) adds the compact shape as one 16-wave
# block per CU (window field 152).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-abc}
mkdir -p "$OUT"
V=${ABC_VARIANTS:-"16,2,2,0,18,1,24:16,2,1,0,18,1,24:16,2,2,0,18,1,56"}
export XSKNF_GPU_LIB=$R/${ABC_LIB:-build/ab}/libxsknf_gpu.so
for rep in 1 2; do
  for W in imix:zero:3 imix:nic:3 570:zero:3 1500:zero:1; do
    IFS=: read -r WL C ROT <<< "$W"
    XSKNF_AB_OCCUPANCY=1 timeout -k 10 200 python "$R/tools/tune.py" --workload "$WL" --checks "$C" --rotate "$ROT" \
      --rounds 7 --variants "$V" 2>> "$OUT/err" \
      | sed "s|^{|{\"rep\": $rep, |" >> "$OUT/ab_compact.jsonl" || { tail -20 "$OUT/err"; exit 1; }
  done
done
python3 - "$OUT/ab_compact.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["checks"], tuple(j["shape"]))].append((j["us"], j["matches_default"]))
for k in sorted(d): print(k, d[k])
PY
grep -h occupancy "$OUT/err" | sort | uniq -c
