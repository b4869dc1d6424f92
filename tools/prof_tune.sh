#!/bin/bash
# rocprofv3 kernel-trace + stats of a tools/tune.py run (GPU box).
#   tools/prof_tune.sh <tag> [tune args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/proftune_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
    -- python3 "$R/tools/tune.py" "$@" > "$OUT/tune.json" 2> "$OUT/stderr.log"
