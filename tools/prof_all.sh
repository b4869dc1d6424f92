#!/bin/bash
# rocprofv3 evidence for bench workloads, summarized on the GPU box (the raw
# traces can exceed gpurun's 64 MiB merge limit) and the raw files deleted:
#   tools/prof_all.sh <tag> <workload>...
# -> gpurun_out/summary_<tag>/{kernels,traffic,bench}_<w>.json, <w>_kernel_stats.csv
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
cd "$R"
SUM=$R/gpurun_out/summary_$TAG
mkdir -p "$SUM"
for W in "$@"; do
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
du -sh gpurun_out
echo "prof_all $TAG done"
