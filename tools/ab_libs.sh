#!/bin/bash
# A/B of alternative builds of the library (XSKNF_GPU_LIB) on the GPU box, each
# lib over several workloads with tools/tune.py, two interleaved repetitions.
#   tools/ab_libs.sh <tag> "<lib1> <lib2> ..." "<wl>:<variants> ..."   (lib "default" = the in-tree build)
set -o pipefail
TAG=$1; LIBS=$2; SPECS=$3
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for L in $LIBS; do
    if [ "$L" = default ]; then unset XSKNF_GPU_LIB; else export XSKNF_GPU_LIB=$PWD/$L; fi
    for spec in $SPECS; do
      wl=${spec%%:*}; vs=${spec#*:}
      echo "== $L $rep $wl" >> gpurun_out/ab/$TAG.txt
      timeout -k 10 120 python tools/tune.py --workload $wl --variants "$vs" --rounds 5 >> gpurun_out/ab/$TAG.txt 2>/dev/null || exit 1
    done
  done
done
grep -v "^$" gpurun_out/ab/$TAG.txt | cut -c1-110
