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
frame) counts 1:1.  A launch is the summing kernel plus the scatter_checks
pass after it (jumbo); a step of more than 1M frames is several launches.

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


def launches(rows):
    """Per launch of the hot path: the summing kernel's value plus that of the
    scatter_checks pass that follows it, if any (jumbo's per-tile policy)."""
    out = []
    for k, v in rows:
        if "scatter_checks" in k and out:
            out[-1] += v
        else:
            out.append(v)
    return out


def class_factor(ln, cal):
    """Counted / true FETCH_SIZE bytes for frames of `ln` bytes (the nearest
    calibrated length of the same kind), or None without a calibration."""
    if not cal:
        return None
    keys = sorted(int(k) for k in cal)
    return cal[str(min(keys, key=lambda k: abs(k - ln)))]


def mixed_factor(bench, workload, cal):
    """The records-only pass's counted / true read bytes, predicted per size
    class from the calibration: sum_c n_c B_c f_c + 16 n f_desc over
    sum_c n_c B_c + 16 n (descriptors: a wide coalesced stream, f = 1/2)."""
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from xsknf_amd import frames
    n = int(bench["config"]["frames_per_gpu"])
    length = bench["config"]["frame_len"]
    if workload == "config4":
        lens = frames.imix_lengths(n, np.random.default_rng(frames.SEED))
    else:
        lens = frames._lens(n, length, np.random.default_rng(frames.SEED))
    vals, cnt = np.unique(lens, return_counts=True)
    true = counted = 0.0
    per = {}
    for v, c in zip(vals.tolist(), cnt.tolist()):
        b = (v + 15) // 16 * 16
        f = class_factor(v, cal)
        true += c * b
        counted += c * b * f
        per[str(v)] = {"frames": c, "factor": f}
    true += 16 * n
    counted += 16 * n * 0.5
    return counted / true, per


def main():
    d, workload = sys.argv[1], sys.argv[2]
    cal = None
    if len(sys.argv) > 3:
        cal = json.load(open(sys.argv[3]))["factors"]
    bench = json.load(open(os.path.join(d, "FETCH_SIZE.bench.json")))
    kalone = bench["roofline"].get("summing_kernel_alone")
    # launches per step: a batch of more than 1M frames runs as 1M-frame launches (config 4 on one GPU)
    # (the lane kernel, frames <= 128 B, takes up to 16M frames per launch)
    # (frame_len is a string for a mix: "imix")
    lane64 = str(bench["config"].get("frame_len")) == "64" and "lane" in bench["roofline"].get("kernels", "")
    per_step = -(-int(bench["config"]["frames_per_gpu"]) // (1 << (24 if lane64 else 20)))
    tail = per_step * (3 + int(bench.get("kernel_steps", 50))) if kalone else 0
    fetch = dispatches(d, "FETCH_SIZE")
    write = dispatches(d, "WRITE_SIZE")
    kernel = ", ".join(sorted({k for k, _ in fetch})) if fetch else None
    f_step, f_rec = split_runs(launches(fetch), tail)
    w_step, w_rec = split_runs(launches(write), tail)
    med = statistics.median
    KiB = 1024
    per_class = None
    if f_rec and cal:
        fmix, per_class = mixed_factor(bench, workload, cal)
        stream = med(f_rec) * KiB / fmix
        rest = max(0.0, med(f_step) - med(f_rec)) * KiB
        fetch_b = stream + rest
        how = (f"FETCH_SIZE of the records-only pass / {fmix:.4f} (its counted/true ratio predicted per size class "
               "from the probe calibration: sum_c n_c B_c f_c over sum_c n_c B_c, descriptors at 1/2) + 1 x the "
               "step's FETCH_SIZE beyond it (the tail's check-sector re-reads: 64-B sectors count 1:1)")
    elif f_rec:
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
        "workload": workload, "kernel": kernel, "launches_per_step": per_step,
        "hbm_bytes_per_step": int((fetch_b + write_b) * per_step),
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "fetch_bytes": int(fetch_b), "write_bytes": int(write_b),
        "fetch_streaming_bytes": int(stream), "fetch_other_bytes": int(rest),
        "records_only_pass": ({"fetch_bytes": int(2 * med(f_rec) * KiB), "write_bytes": int(med(w_rec) * KiB)}
                              if f_rec else None),
        "raw_KiB": {"fetch_step_median": med(f_step), "fetch_records_only_median": med(f_rec) if f_rec else None,
                    "write_step_median": write_b / KiB, "step_dispatches": len(f_step)},
        "alg_bytes_per_step": bench["roofline"]["alg_bytes_per_step"],
        "size_classes": per_class,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; " + how +
                  "; write = WRITE_SIZE; medians per dispatch",
    }
    out["traffic_over_alg"] = round(out["hbm_bytes_per_step"] / out["alg_bytes_per_step"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
