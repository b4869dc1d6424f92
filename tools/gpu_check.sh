#!/bin/bash
# One GPU-box pass: parity tests, the bench (all workloads), smoke (run ON the GPU box).
#   tools/gpu_check.sh [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-check}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 400 python bench.py > "$OUT/bench_all.json" 2> "$OUT/bench_all.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench_all.err"; exit 1; }
cat "$OUT/bench_all.json"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
