#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 --pmc counter_collection.csv.

usage: pmc_summary.py <dir or *_counter_collection.csv> [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "*counter_collection.csv"))[0]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(path) as f:
        for r in csv.DictReader(f):
            if flt and flt not in r["Kernel_Name"]:
                continue
            agg[r["Kernel_Name"][:48]][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for d in agg.values() for c in d})
    for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        print(k)
        for c in names:
            if c in d:
                print("   %-24s %14.4g" % (c, d[c]))


if __name__ == "__main__":
    main()
