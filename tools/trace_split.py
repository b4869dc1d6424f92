#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of bench.py into the summing kernel's launches
inside a step (followed by scatter_checks) and launched alone (the bench's
records-only roofline leg); prints JSON with count / mean / median in us.

    python tools/trace_split.py gpurun_out/prof_<tag>/run_kernel_trace.csv
"""
import csv
import json
import statistics as st
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
           for r in rows if "xsknf_gpu::" in r["Kernel_Name"]]
    legs = {"checksum_kernel in step": [], "checksum_kernel alone (records only)": [], "scatter_checks": []}
    for i, (name, us) in enumerate(seq):
        if "scatter_checks" in name:
            legs["scatter_checks"].append(us)
        elif "checksum_kernel" in name:
            nxt = seq[i + 1][0] if i + 1 < len(seq) else ""
            legs["checksum_kernel in step" if "scatter_checks" in nxt else
                 "checksum_kernel alone (records only)"].append(us)
    out = {k: {"launches": len(v), "mean_us": round(st.mean(v), 2), "median_us": round(st.median(v), 2)}
           for k, v in legs.items() if v}
    out["kernel"] = next((n for n, _ in seq if "checksum_kernel" in n), None)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
