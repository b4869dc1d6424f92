#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration on known byte counts (measurement infra).

tools/prof_round.sh runs rocprofv3 --pmc over tools/build/hbm_probe reading
1,048,576 frames of LEN bytes at a 2 KiB stride (data at +256) -- the aligned
UMEM pattern of each IMIX size class.  The guide (MI355X_MICROARCH.md, HBM)
says FETCH_SIZE reports half of a wide coalesced streaming read and that other
access widths must be calibrated in one's own pattern: this writes the factor
counted / true bytes per LEN, which tools/traffic.py divides out per class.

    python tools/pmc_calib.py gpurun_out/pmc_<tag>_calib > profiles/r03/pmc_calibration.json
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

N = 1 << 20


def kib_per_dispatch(d, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return statistics.median(vals) if vals else None, len(vals)


def main():
    d = sys.argv[1]
    out = {"pattern": "1,048,576 frames at a 2048-B stride, data at +256, read in 16-B pieces by tools/build/hbm_probe",
           "factors": {}, "raw": {}}
    for sub in sorted(glob.glob(os.path.join(d, "FETCH_SIZE_*"))):
        if not os.path.isdir(sub):
            continue
        ln = int(re.search(r"_(\d+)$", sub).group(1))
        kib, nd = kib_per_dispatch(sub, "FETCH_SIZE")
        if kib is None:
            continue
        true = N * ((ln + 15) // 16 * 16)
        out["raw"][str(ln)] = {"FETCH_SIZE_KiB_per_dispatch": kib, "dispatches": nd, "true_bytes": true}
        out["factors"][str(ln)] = round(kib * 1024 / true, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
