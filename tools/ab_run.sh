#!/bin/bash
# A/B of launch shapes on the GPU box (tools/tune.py; one process per workload)
#   tools/ab_run.sh <tag> <workload>:<variants> ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/ab
for spec in "$@"; do
  wl=${spec%%:*}; vs=${spec#*:}
  echo "== $wl" >> gpurun_out/ab/$TAG.txt
  timeout -k 10 150 python tools/tune.py --workload $wl --variants "$vs" --rounds 7 >> gpurun_out/ab/$TAG.txt 2>/dev/null || exit 1
done
cat gpurun_out/ab/$TAG.txt
