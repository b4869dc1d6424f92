#!/bin/bash
# Round-3 evidence for the NIC-checksum workloads (run ON the GPU box):
#   tools/prof_nic.sh <tag>
# rocprofv3 kernel stats and FETCH_SIZE / WRITE_SIZE passes of the bench's
# *-nic workloads, summarized on the box (tools/prof_summary.py,
# tools/traffic.py) and the raw traces deleted (the frame generator's torch
# kernels make them large); then the end-to-end host path and the NF-level
# hook rates on NIC-checksummed frames.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-nic}
cd "$R"
SUM=$R/gpurun_out/summary_$TAG
mkdir -p "$SUM"
for W in 1500-nic imix-nic 64-nic jumbo-nic; do
  "$R/tools/prof_stats.sh" "${TAG}_$W" --workload $W || { echo "prof $W failed"; exit 1; }
  D=$R/gpurun_out/prof_${TAG}_$W
  python3 tools/prof_summary.py "$D" > "$SUM/kernels_$W.json" || { echo "summary $W failed"; exit 1; }
  cp "$D/bench.json" "$SUM/bench_$W.json"
  find "$D" -name '*kernel_stats.csv' -exec cp {} "$SUM/${W}_kernel_stats.csv" \;
  rm -rf "$D"
  "$R/tools/prof_pmc.sh" "${TAG}_$W" --workload $W || { echo "pmc $W failed"; exit 1; }
  P=$R/gpurun_out/pmc_${TAG}_$W
  python3 tools/traffic.py "$P" $W profiles/r03/pmc_calibration.json > "$SUM/traffic_$W.json" \
    || { echo "traffic $W failed"; exit 1; }
  rm -rf "$P"
done
mkdir -p gpurun_out/e2e_$TAG
for C in nic zero; do
  timeout -k 10 300 python tools/e2e_bench.py --checks $C --check --orders rx,scattered --modes async \
      --batches 1024,16384,1048576 --seconds 1.5 > gpurun_out/e2e_$TAG/e2e_$C.jsonl 2>&1 || { echo "e2e $C failed"; exit 1; }
done
HOOK_BENCH_CHECKS=nic "$R/tools/hook_bench.sh" hook_${TAG} > /dev/null || { echo "hook_bench nic failed"; exit 1; }
du -sh gpurun_out
echo "prof_nic $TAG done"
