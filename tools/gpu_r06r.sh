set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r06r}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --secondary "" --cpu-seconds 0 --no-probes > $OUT/bench.json 2> $OUT/bench.err || { echo prof failed; tail -20 $OUT/bench.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
python3 - "$OUT" <<'PY'
import csv, sys, os, json
out = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(out, "kernel_stats.csv"))))
keep = [r for r in rows if any(k in r["Name"] for k in ("pack_frames", "apply_records", "shard_counters", "checksum_kernel"))]
json.dump(keep, open(os.path.join(out, "multi_kernels.json"), "w"), indent=1)
for r in keep:
    print(r["Name"][:90], r["Calls"], r["AverageNs"])
PY
find $OUT/prof -name '*kernel_trace.csv' -size +20M -delete
