#!/bin/bash
# Interleaved A/B matrix on the GPU box (tools/tune.py, one process per case):
#   tools/ab_matrix.sh <tag> <reps> <case> ...
# case = lib:workload:checks:rotate[:variants]   (lib: "lib" = the product
# library, else build/<lib>/; variants as tune.py --variants, ';' for ':')
# -> gpurun_out/<tag>/ab.jsonl and a summary (median per case of the runs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$1; REPS=$2; shift 2
mkdir -p "$OUT"
for rep in $(seq 1 $REPS); do
  for c in "$@"; do
    IFS=: read L W C K V <<< "$c"
    LIB=$R/build/$L/libxsknf_gpu.so; [ $L = lib ] && LIB=$R/xsknf_amd/lib/libxsknf_gpu.so
    XSKNF_GPU_LIB=$LIB timeout -k 10 200 python "$R/tools/tune.py" --workload $W --checks $C --rotate $K \
      --rounds 5 ${V:+--variants "${V//;/:}"} 2>> "$OUT/err" \
      | sed "s|^{|{\"lib\": \"$L\", \"rep\": $rep, |" >> "$OUT/ab.jsonl" || { tail -20 "$OUT/err"; exit 1; }
  done
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    d[(j["workload"], j["checks"], j["lib"], ",".join(map(str, j["shape"])), j["matches_default"])].append(j["us"])
for k in sorted(d): print(k, sorted(d[k]))
PY
