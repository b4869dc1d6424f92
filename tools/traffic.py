#!/usr/bin/env python3
"""HBM traffic per hot-path step from rocprofv3 --pmc passes (tools/prof_pmc.sh).

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports exactly half of
the bytes of a wide coalesced streaming read, so the summing kernel's fetched
bytes = 2 x FETCH_SIZE (KiB); the scatter pass's sector / word reads are taken
1:1 (they match its byte count); WRITE_SIZE reads bytes exactly for 16-B
streaming stores.
A step of the hot path = the summing kernel + the scatter kernel; their
per-dispatch means are added.

    python tools/traffic.py gpurun_out/pmc_<tag> <workload> > profiles/traffic_<workload>.json
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("checksum_kernel", "scatter_checks")


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            for k in KERNELS:
                if k in name:
                    acc[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items() if v}


def main():
    d, workload = sys.argv[1], sys.argv[2]
    fetch = per_kernel(d, "FETCH_SIZE")
    write = per_kernel(d, "WRITE_SIZE")
    # the 2x correction holds for wide coalesced streaming reads (the summing
    # kernel); the scatter pass reads 64-B sectors and 4-16 B words, counted 1:1
    fetch_b = sum((2 if "checksum_kernel" in k else 1) * 1024 * v for k, v in fetch.items())
    write_b = sum(1024 * v for v in write.values())
    # the dominant kernel alone (bench.py's roofline.traffic): the summing kernel
    sk = [k for k in fetch if "checksum_kernel" in k]
    dom = None
    if sk:
        k = max(sk, key=lambda k: fetch[k])
        dom = {"kernel": k, "hbm_bytes_per_launch": int(2 * 1024 * fetch[k] + 1024 * write.get(k, 0.0))}
    out = {
        "workload": workload,
        "dominant": dom,
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "fetch_bytes": int(fetch_b), "write_bytes": int(write_b),
        "per_kernel_fetch_KiB_raw": fetch, "per_kernel_write_KiB_raw": write,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; "
                  "fetch = 2 x FETCH_SIZE for the streaming summing kernel (gfx950 half-count "
                  "correction), 1 x for the scatter pass; write = WRITE_SIZE; "
                  "per dispatch, summing + scatter kernels of one step",
    }
    print(json.dumps(out, indent=1))


def add_dominant(path):
    """Add the `dominant` entry to an existing traffic_<workload>.json."""
    d = json.load(open(path))
    fetch, write = d["per_kernel_fetch_KiB_raw"], d["per_kernel_write_KiB_raw"]
    k = max((k for k in fetch if "checksum_kernel" in k), key=lambda k: fetch[k])
    d["dominant"] = {"kernel": k, "hbm_bytes_per_launch": int(2 * 1024 * fetch[k] + 1024 * write.get(k, 0.0))}
    json.dump(d, open(path, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--add-dominant":
        add_dominant(sys.argv[2])
    else:
        main()
