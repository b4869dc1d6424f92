#!/bin/bash
# Dynamic vs static tile schedule of the split kernel (run ON the GPU box):
#   tools/ab_dyn.sh <tag> [libdir ...]
# fused_stores 18 = the product (dynamic schedule), 50 = 18 + 32 (static).
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
for L in ${@:-xsknf_amd/lib}; do
  for W in 1500 570 imix 1024; do
    R=1; [ $W = imix ] && R=4; [ $W = 570 ] && R=2
    XSKNF_GPU_LIB=$PWD/$L/libxsknf_gpu.so timeout -k 10 150 python tools/tune.py --workload $W --rotate $R --bpc 4 \
      --rounds 6 --variants ${VARIANTS:-16,2,2,0,50,1,24} 2>>"$OUT/err" | sed "s|^{|{\"lib\": \"$L\", |" >> "$OUT/res.jsonl" || exit 1
  done
done
cut -c1-200 "$OUT/res.jsonl"
