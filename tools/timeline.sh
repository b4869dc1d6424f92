#!/bin/bash
# Per-wave timelines of the split kernel (run ON the GPU box after `make tl`):
#   tools/timeline.sh <tag> [workload[:variant] ...]
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for WV in ${@:-1500 570 imix}; do
  W=${WV%%:*}; V=""; [ "$W" != "$WV" ] && V="--variant ${WV#*:}"
  R=1; [ $W = imix ] && R=4; [ $W = 570 ] && R=2
  XSKNF_GPU_LIB=$PWD/${TL_LIB:-build/tl}/libxsknf_gpu.so timeout -k 10 120 python tools/timeline.py --workload $W --rotate $R $V \
    >> "$OUT/timeline.jsonl" 2>>"$OUT/err" || { tail -20 "$OUT/err"; exit 1; }
done
cat "$OUT/timeline.jsonl"
