#!/bin/bash
# Interleaved A/B of N builds of libxsknf_gpu on the default shapes (tools/tune.py):
#   tools/ab_n_libs.sh <tag> "<libdir> <libdir> ..." [rounds] [workloads]   (run ON the GPU box)
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
WLS=${4:-"1500 imix 570"}
for r in $(seq 1 ${3:-2}); do
  for L in $2; do
    for W in $WLS; do
      R=1; [ $W = imix ] && R=4; [ $W = 570 ] && R=2; [ $W = 64 ] && R=13
      XSKNF_GPU_LIB=$PWD/$L/libxsknf_gpu.so timeout -k 10 100 python tools/tune.py --workload $W --rotate $R --bpc 4 \
        --rounds 5 2>>"$OUT/err" | sed "s|^{|{\"lib\": \"$L\", |" >> "$OUT/res.jsonl" || exit 1
    done
  done
done
python3 - "$OUT/res.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l); d[(j["workload"], j["lib"])].append(j["us"])
for k in sorted(d): print(k, d[k])
PY
