#!/usr/bin/env python3
"""HBM traffic per hot-path step from rocprofv3 --pmc passes (tools/prof_pmc.sh).

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports exactly half of
the bytes of a wide coalesced streaming read, so fetched bytes = 2 x FETCH_SIZE
(KiB); WRITE_SIZE reads bytes exactly for 16-B-per-lane streaming stores.
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
    fetch_b = sum(2 * 1024 * v for v in fetch.values())
    write_b = sum(1024 * v for v in write.values())
    out = {
        "workload": workload,
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "fetch_bytes": int(fetch_b), "write_bytes": int(write_b),
        "per_kernel_fetch_KiB_raw": fetch, "per_kernel_write_KiB_raw": write,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; "
                  "fetch = 2 x FETCH_SIZE (gfx950 half-count correction), write = WRITE_SIZE; "
                  "per dispatch, summing + scatter kernels of one step",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
