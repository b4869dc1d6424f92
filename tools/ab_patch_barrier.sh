#!/bin/bash
# A/B (round 3): a grid-wide barrier before the per-wave patches (fused_stores + 64)
# hypothesis: the sector writes cost ~31 us beside the other blocks' streams and
# ~20 us after them (probe_mix); stop rule: keep at >= 4 us gain at 1500 B worst
# case, no loss at IMIX / NIC
set -o pipefail
export XSKNF_GPU_LIB=build/ab/libxsknf_gpu.so
mkdir -p gpurun_out/ab
for rep in 1 2; do
  timeout -k 10 200 python tools/tune.py --workload 1500 --checks zero --rounds 7 \
      --variants "16,2,2,0,82,1,56" >> gpurun_out/ab/ab_patch_barrier.txt || exit 1
  timeout -k 10 200 python tools/tune.py --workload imix --checks zero --rotate 3 --rounds 7 \
      --variants "16,2,2,0,82,1,24" >> gpurun_out/ab/ab_patch_barrier.txt || exit 1
  timeout -k 10 200 python tools/tune.py --workload 570 --checks zero --rounds 7 \
      --variants "16,2,2,0,82,1,56" >> gpurun_out/ab/ab_patch_barrier.txt || exit 1
done
