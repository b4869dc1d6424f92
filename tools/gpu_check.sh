#!/bin/bash
# One GPU-box pass: parity tests, the bench (all workloads), smoke (run ON the GPU box).
#   tools/gpu_check.sh [tag] [--starts N]
# --starts N first runs tools/nf_start_probe.py (N NF-shaped process starts in
# the GPU suite's shape, DESIGN 3 "NF start").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-check}
STARTS=0
[ "$2" = "--starts" ] && STARTS=$3
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
if [ "$STARTS" -gt 0 ]; then
    timeout -k 10 400 python -u tools/nf_start_probe.py --starts "$STARTS" --out "$OUT/nf_start_probe.jsonl" \
        > "$OUT/nf_start_probe.log" 2>&1 || { echo "start probe failed"; tail -30 "$OUT/nf_start_probe.log"; exit 1; }
    tail -2 "$OUT/nf_start_probe.log"
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
cp gpurun_out/nf_starts.jsonl "$OUT/" 2>/dev/null
timeout -k 10 400 python bench.py > "$OUT/bench_all.json" 2> "$OUT/bench_all.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench_all.err"; exit 1; }
cat "$OUT/bench_all.json"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
