#!/usr/bin/env python3
"""Per-kernel durations of one bench.py run under rocprofv3 --kernel-trace
(tools/prof_stats.sh), split the way the bench dispatches them:

  * the step's kernels (warm-up + timed steps, and a scatter_checks launch per
    step where the shape has one) -- the last --steps of them are the timed ones;
  * the split kernel again in records-only mode (the summing pass alone,
    bench.py's `summing_kernel_alone`): the last 3 + --kernel-steps dispatches.

Prints the mean / median duration of each, to compare with the bench line's
HIP-event figures (roofline.step_us, summing_kernel_alone.us).

    python tools/prof_summary.py gpurun_out/prof_<tag> > profiles/<round>/kernels_<workload>.json
"""
import csv
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    bench = json.load(open(os.path.join(d, "bench.json")))
    steps = int(bench["steps"])
    kalone = bench["roofline"].get("summing_kernel_alone") is not None
    rows = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        if "xsknf_gpu::" in r["Kernel_Name"]:
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows.sort()
    main_name = rows[0][1]
    # a batch of more than 1M frames runs as 1M-frame launches (config 4 on one GPU)
    # (the lane kernel, frames <= 128 B, takes up to 16M frames per launch)
    # (frame_len is a string for a mix: "imix")
    lane64 = str(bench["config"].get("frame_len")) == "64" and "lane" in bench["roofline"].get("kernels", "")
    per_step = -(-int(bench["config"]["frames_per_gpu"]) // (1 << (24 if lane64 else 20)))
    ksteps = int(bench.get("kernel_steps", 50))
    tail = per_step * (3 + ksteps) if kalone else 0
    mains = [r for r in rows if r[1] == main_name]
    step_main = mains[:len(mains) - tail] if tail else mains
    alone = mains[len(mains) - tail:] if tail else []
    scatter = [r for r in rows if "scatter_checks" in r[1]]
    timed = step_main[-steps * per_step:]
    out = {"bench_step_us": bench["roofline"]["step_us"],
           "bench_summing_alone_us": (bench["roofline"]["summing_kernel_alone"] or {}).get("us"),
           "kernel": main_name, "launches_per_step": per_step,
           "step_kernel_us": {"mean": round(statistics.mean(r[2] for r in timed), 2),
                              "median": round(statistics.median(r[2] for r in timed), 2), "n": len(timed)}}
    per_launch = statistics.mean(r[2] for r in timed)
    if scatter:
        ts = scatter[-steps * per_step:]
        out["scatter_checks_us"] = {"mean": round(statistics.mean(r[2] for r in ts), 2),
                                    "median": round(statistics.median(r[2] for r in ts), 2), "n": len(ts)}
        per_launch += statistics.mean(r[2] for r in ts)
    # the step from the trace: its launches' kernel durations (gaps between kernels excluded)
    out["trace_step_us"] = round(per_step * per_launch, 2)
    if alone:
        a = alone[3 * per_step:]
        out["records_only_us"] = {"mean": round(statistics.mean(r[2] for r in a), 2),
                                  "median": round(statistics.median(r[2] for r in a), 2), "n": len(a)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
