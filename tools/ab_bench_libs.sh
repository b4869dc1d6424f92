#!/bin/bash
# A/B of library builds through bench.py itself (the headline's own method:
# rotation, -i 1/2 alternation, warmup), libraries interleaved, REPS rounds:
#   tools/ab_bench_libs.sh <tag> "<lib dir> ..." [secondaries] [reps]
# ("xsknf_amd/lib" = the product build) -> gpurun_out/ab/<tag>_bench.jsonl
set -o pipefail
TAG=$1; LIBS=$2; SEC=${3:-imix}; REPS=${4:-3}
mkdir -p gpurun_out/ab
for rep in $(seq "$REPS"); do
  for L in $LIBS; do
    XSKNF_GPU_LIB=$PWD/$L/libxsknf_gpu.so timeout -k 10 300 python bench.py --secondary "$SEC" --cpu-seconds 0 \
      --no-probes 2> gpurun_out/ab/${TAG}_bench.err | grep '^{' | sed "s|^{|{\"lib\": \"$L\", \"rep\": $rep, |" \
      >> gpurun_out/ab/${TAG}_bench.jsonl || { tail -20 gpurun_out/ab/${TAG}_bench.err; exit 1; }
  done
done
python3 - gpurun_out/ab/${TAG}_bench.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    j = json.loads(l)
    d[("1500", j["lib"])].append(round(j["ms_per_step"] * 1e3, 1))
    for k, v in j.get("secondary", {}).items():
        d[(k, j["lib"])].append(v.get("step_us"))
for k in sorted(d): print(k, d[k])
PY
