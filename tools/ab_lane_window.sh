#!/bin/bash
# A/B (needs `make ab`): the lane kernel's window, 5 chunks (default) vs 4,
# on 64 B / 60 B frames, aligned and unaligned (odd starts), worst case
# (every check changes) and NIC-checksummed traffic:
#   tools/ab_lane_window.sh <tag>  -> gpurun_out/<tag>/ab_lane_window.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/${1:-ablw}
mkdir -p "$OUT"
export XSKNF_GPU_LIB=$R/build/ab/libxsknf_gpu.so
for W in 64 64u 60 60u; do
  for C in nic zero; do
    timeout -k 10 200 python "$R/tools/tune.py" --workload $W --checks $C --rotate 13 --rounds 7 \
      --variants "1,4,2,0,1:1,4,1,0,1:1,5,1,0,1:1,4,1,0,1,0,160" >> "$OUT/ab_lane_window.jsonl" 2>> "$OUT/err" \
      || { tail -20 "$OUT/err"; exit 1; }
  done
done
cat "$OUT/ab_lane_window.jsonl"
