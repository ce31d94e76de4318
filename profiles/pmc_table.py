#!/usr/bin/env python3
"""Per-kernel SQ counter table (per wave) from a rocprofv3 --pmc counter_collection.csv.

usage: pmc_table.py <dir or *_counter_collection.csv> [top-n]
WAVE_CYCLES / WAIT_* / ACTIVE_INST_ANY are quad-cycles (x4 = shader cycles).
"""
import collections
import csv
import glob
import os
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, "*counter_collection.csv"))[0]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 16
agg = collections.defaultdict(lambda: collections.defaultdict(float))
with open(path) as f:
    for r in csv.DictReader(f):
        agg[r["Kernel_Name"].replace("void ", "")[:34]][r["Counter_Name"]] += float(r["Counter_Value"])
cols = sorted({c for d in agg.values() for c in d} - {"SQ_WAVES"})
print("%-34s %9s" % ("kernel", "waves") + "".join("%12s" % c[3:15] for c in cols) + "   (per wave)")
for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:top]:
    n = max(d.get("SQ_WAVES", 1), 1)
    print("%-34s %9.3g" % (k, n) + "".join("%12.0f" % (d[c] / n) for c in cols))
