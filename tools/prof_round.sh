#!/bin/bash
# The round's GPU evidence in one call (run ON the GPU box):
#   tools/prof_round.sh <tag>
# parity tests + smoke + bench (1500 primary, all secondaries), one bench line
# per workload as primary, rocprofv3 kernel stats of the 1500 / IMIX / 64 B
# benches, and the FETCH_SIZE / WRITE_SIZE passes of the 1500 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-round}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
"$R/tools/gpu_check.sh" "$TAG" || exit 1
cd "$R"
for W in 64 imix jumbo; do
  timeout -k 10 240 python bench.py --workload $W --secondary "" > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" \
      || { echo "bench $W failed"; tail -20 "$OUT/bench_$W.err"; exit 1; }
done
"$R/tools/prof_stats.sh" "${TAG}_1500" || { echo "prof 1500 failed"; exit 1; }
"$R/tools/prof_stats.sh" "${TAG}_imix" --workload imix || { echo "prof imix failed"; exit 1; }
"$R/tools/prof_stats.sh" "${TAG}_64" --workload 64 || { echo "prof 64 failed"; exit 1; }
"$R/tools/prof_pmc.sh" "${TAG}_1500" || { echo "pmc 1500 failed"; exit 1; }
echo "prof_round $TAG done"
