#!/bin/bash
# Why the default bench line's secondary.jumbo reads ~20 us above jumbo timed
# alone: the same bench with the workloads before it and the probes on or off.
#   tools/ab_jumbo_warmup.sh <tag> [probes|order|cache|lane13m]   (ON the GPU box) -> gpurun_out/<tag>/ab.jsonl
set -o pipefail
OUT=gpurun_out/${1:-r05jw}; mkdir -p "$OUT"
run() {   # case args...
  local c=$1; shift
  timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" 2>>"$OUT/err" | grep '^{' \
    | sed "s|^{|{\"case\": \"$c\", \"rep\": $rep, |" >> "$OUT/ab.jsonl"
}
CASES=${2:-probes}
for rep in 1 2; do
  if [ "$CASES" = probes ]; then
    export XSKNF_BENCH_EMPTY_CACHE=1   # (recorded with the round-4 behaviour)
    run A-64-imix-jumbo-noprobes --secondary 64,imix,jumbo --no-probes || exit 1
    run B-64-imix-jumbo-probes --secondary 64,imix,jumbo || exit 1
    run C-jumbo-probes --secondary jumbo || exit 1
  elif [ "$CASES" = cache ]; then   # the freed memory kept in torch's cache, and config 4 by order
    run G-64-imix-jumbo-config4-keepcache --secondary 64,imix,jumbo,config4 --no-probes || exit 1
    XSKNF_BENCH_EMPTY_CACHE=1 run H-64-imix-jumbo-config4 --secondary 64,imix,jumbo,config4 --no-probes || exit 1
    run I-jumbo-config4-64-imix --secondary jumbo,config4,64,imix --no-probes || exit 1
  elif [ "$CASES" = lane13m ]; then   # the 13M-frame lane batch after the 64 B workload, cache kept or not
    run J-64-13M-keepcache --secondary 64,64-13M --no-probes || exit 1
    XSKNF_BENCH_EMPTY_CACHE=1 run K-64-13M-emptycache --secondary 64,64-13M --no-probes || exit 1
    run L-13M-alone --secondary 64-13M --no-probes || exit 1
  else   # which workload before it
    export XSKNF_BENCH_EMPTY_CACHE=1   # (recorded with the round-4 behaviour)
    run D-64-jumbo --secondary 64,jumbo --no-probes || exit 1
    run E-imix-jumbo --secondary imix,jumbo --no-probes || exit 1
    run F-jumbo-64-imix --secondary jumbo,64,imix --no-probes || exit 1
  fi
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    j = json.loads(l); s = j.get("secondary", {})
    print(j["case"], j["rep"], {k: v["step_us"] for k, v in s.items()})
PY
