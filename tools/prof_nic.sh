#!/bin/bash
# Round-3 evidence for the NIC-checksum workloads (run ON the GPU box):
#   tools/prof_nic.sh <tag>
# rocprofv3 kernel stats and FETCH_SIZE / WRITE_SIZE passes of the bench's
# *-nic workloads, then the end-to-end host path on NIC-checksummed and on
# zero-check frames.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-nic}
cd "$R"
for W in 1500-nic imix-nic 64-nic jumbo-nic; do
  "$R/tools/prof_stats.sh" "${TAG}_$W" --workload $W || { echo "prof $W failed"; exit 1; }
done
for W in 1500-nic imix-nic 64-nic jumbo-nic; do
  "$R/tools/prof_pmc.sh" "${TAG}_$W" --workload $W || { echo "pmc $W failed"; exit 1; }
done
mkdir -p gpurun_out/e2e_$TAG
for C in nic zero; do
  timeout -k 10 300 python tools/e2e_bench.py --checks $C --check --orders rx,scattered --modes async \
      --batches 1024,16384,1048576 --seconds 1.5 > gpurun_out/e2e_$TAG/e2e_$C.jsonl 2>&1 || { echo "e2e $C failed"; exit 1; }
done
echo "prof_nic $TAG done"
