#!/bin/bash
# A/B (round 3): 1500 B launch shapes now that the suite fault is explained
# (the 16 x 3 static shape left the product over it in round 2)
set -o pipefail
export XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so
mkdir -p gpurun_out/ab
for ch in zero nic zero; do
  timeout -k 10 200 python tools/tune.py --workload 1500 --checks $ch --rounds 7 \
      --variants "16,3,2,0,18,1,24:16,3,2,0,18,1,52:16,2,2,0,18,1,24" >> gpurun_out/ab/ab_1500_shapes.txt || exit 1
done
