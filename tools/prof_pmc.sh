#!/bin/bash
# HBM traffic counters of one bench workload, one rocprofv3 --pmc pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
#   tools/prof_pmc.sh <tag> [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o run \
      -- python3 "$R/bench.py" --cpu-seconds 0 --no-probes --no-c-host-multi --secondary "" "$@" > "$OUT/$C.bench.json" 2> "$OUT/$C.stderr.log"
done
