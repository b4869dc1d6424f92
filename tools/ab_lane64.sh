#!/bin/bash
# A/B (round 3): lane-kernel windows at 64 B, NIC checks and zero checks, more rounds
set -o pipefail
export XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so
mkdir -p gpurun_out/ab
for ch in nic zero nic zero; do
timeout -k 10 200 python tools/tune.py --workload 64 --checks $ch --rotate 13 --rounds 9 \
    --variants "1,4,2,0,1:1,4,1,0,1:1,4,1,0,1,0,160" >> gpurun_out/ab/ab_lane64.txt || exit 1
done
