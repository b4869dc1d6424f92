#!/usr/bin/env python3
"""HBM traffic per hot-path step from rocprofv3 --pmc passes (tools/prof_pmc.sh).

A bench.py run dispatches the step's kernel (warm-up + timed steps) and then,
for the split kernel, the same kernel in records-only mode (the summing pass
alone: --kernel-steps launches at the end).  Counter calibration (gfx950,
MI355X_MICROARCH.md "HBM"; checked on tools/hbm_probe over known byte counts,
tools/prof_round.sh's calib passes):
  * FETCH_SIZE counts HALF the bytes of a wide coalesced streaming read
    (1M x 1504 B frames: 814,622 KiB = 0.53 x the bytes) -> x 2;
  * 64-byte sector reads (1M x 64 B at a 2 KiB stride) count 1:1 (65,596 KiB);
  * WRITE_SIZE counts streaming and sector stores exactly.
So for the split kernel the streaming share of a step's FETCH_SIZE is the
records-only pass's (x 2), and the rest -- the tail's record / descriptor /
sector re-reads -- counts 1:1; the lane kernel (64 B frames, one sector per
frame) counts 1:1.  All values per dispatch.

    python tools/traffic.py gpurun_out/pmc_<tag>_<workload> <workload> > profiles/traffic_<workload>.json
"""
import csv
import glob
import json
import os
import statistics
import sys

PRODUCT = "xsknf_gpu::"


def dispatches(d, counter):
    """[(kernel, value KiB)] of the product's kernels in dispatch order."""
    rows = []
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and PRODUCT in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    return [(k, v) for _, k, v in rows]


def split_runs(vals, tail):
    """(step dispatches, records-only dispatches): the last `tail` are records-only."""
    if tail and len(vals) > tail:
        return vals[:-tail], vals[-tail:]
    return vals, []


def main():
    d, workload = sys.argv[1], sys.argv[2]
    bench = json.load(open(os.path.join(d, "FETCH_SIZE.bench.json")))
    kalone = bench["roofline"].get("summing_kernel_alone")
    tail = (3 + int(bench.get("kernel_steps", 50))) if kalone else 0
    fetch = dispatches(d, "FETCH_SIZE")
    write = dispatches(d, "WRITE_SIZE")
    kernel = fetch[0][0] if fetch else None
    f_step, f_rec = split_runs([v for _, v in fetch], tail)
    w_step, w_rec = split_runs([v for _, v in write], tail)
    med = statistics.median
    KiB = 1024
    if f_rec:
        stream = 2 * med(f_rec) * KiB
        rest = max(0.0, med(f_step) - med(f_rec)) * KiB
        fetch_b = stream + rest
        how = ("2 x FETCH_SIZE of the records-only pass (streaming) + 1 x the step's FETCH_SIZE beyond it "
               "(tail re-reads of records, descriptors, check sectors)")
    else:
        stream, rest = 0.0, med(f_step) * KiB
        fetch_b = rest
        how = "1 x FETCH_SIZE (one 64-byte sector per frame, calibrated 1:1)"
    write_b = med(w_step) * KiB
    out = {
        "workload": workload, "kernel": kernel,
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "fetch_bytes": int(fetch_b), "write_bytes": int(write_b),
        "fetch_streaming_bytes": int(stream), "fetch_other_bytes": int(rest),
        "records_only_pass": ({"fetch_bytes": int(2 * med(f_rec) * KiB), "write_bytes": int(med(w_rec) * KiB)}
                              if f_rec else None),
        "raw_KiB": {"fetch_step_median": med(f_step), "fetch_records_only_median": med(f_rec) if f_rec else None,
                    "write_step_median": write_b / KiB, "step_dispatches": len(f_step)},
        "alg_bytes_per_step": bench["roofline"]["alg_bytes_per_step"],
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; " + how +
                  "; write = WRITE_SIZE; medians per dispatch",
    }
    out["traffic_over_alg"] = round(out["hbm_bytes_per_launch"] / out["alg_bytes_per_step"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
