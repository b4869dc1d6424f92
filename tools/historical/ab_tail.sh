#!/bin/bash
# A/B of tail-patch batching (XSKNF_PATCH_T builds; the XSKNF_TAIL_TILES record path is gone) on the 1500 B and IMIX steps (run ON the GPU box).
set -o pipefail
cd $GRAFT_REPO_ROOT
for R in 1 2; do
for L in ab ab_t4 ab_t6; do
export XSKNF_GPU_LIB=$GRAFT_REPO_ROOT/build/$L/libxsknf_gpu.so
timeout -k 10 300 python tools/tune.py --workload 1500 --rounds 5 --bpc 8 --variants "16,3,2,0,18,1,24" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$L', d['workload'], d['shape'], d['us'])" || exit 1
timeout -k 10 300 python tools/tune.py --workload imix --rotate 3 --rounds 5 --bpc 8 --variants "16,3,2,0,18,1,24" | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$L', d['workload'], d['shape'], d['us'])" || exit 1
done; done
