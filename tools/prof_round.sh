#!/bin/bash
# The round's profiling evidence in one call (run ON the GPU box):
#   tools/prof_round.sh <tag>
# rocprofv3 kernel stats of the 1500 / IMIX / 64 B / jumbo / config-4 benches,
# their FETCH_SIZE / WRITE_SIZE passes, and the same counters on
# tools/hbm_probe over known byte counts of the 1500 B, 570 B and 64 B access
# patterns (the counters' calibration per IMIX size class, tools/pmc_calib.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-round}
cd "$R"
for W in 1500 imix 64 jumbo config4; do
  "$R/tools/prof_stats.sh" "${TAG}_$W" --workload $W || { echo "prof $W failed"; exit 1; }
done
for W in 1500 imix 64 jumbo config4; do
  "$R/tools/prof_pmc.sh" "${TAG}_$W" --workload $W || { echo "pmc $W failed"; exit 1; }
done
OUT=$R/gpurun_out/pmc_${TAG}_calib
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  for P in "1048576 2048 256 1504" "1048576 2048 256 576" "1048576 2048 256 64"; do
    tag=$(echo $P | awk '{print $4}')
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/${C}_$tag" -o run \
      -- "$R/tools/build/hbm_probe" $P 5 > "$OUT/${C}_$tag.log" 2>&1 || { echo "calib $C $tag failed"; exit 1; }
  done
done
echo "prof_round $TAG done"
