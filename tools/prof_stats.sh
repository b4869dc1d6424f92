#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench workload (run ON the GPU box).
#   tools/prof_stats.sh <tag> [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
    -- python3 "$R/bench.py" --cpu-seconds 0 --no-probes --no-c-host-multi --secondary "" "$@" > "$OUT/bench.json" 2> "$OUT/stderr.log"
