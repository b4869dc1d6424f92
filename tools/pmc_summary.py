#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel name, mean counter value per dispatch."""
import collections
import csv
import glob
import os
import sys


def summarise(d, match=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if match and match not in name:
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


if __name__ == "__main__":
    for d in sys.argv[1:]:
        for name, cs in summarise(d).items():
            print(f"{d} :: {name[:80]}")
            for c, v in sorted(cs.items()):
                print(f"   {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")
