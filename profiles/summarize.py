#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory.

usage: summarize.py <rocprofv3 output dir or *_kernel_stats.csv> [launches]

Prints kernels by total time; with `launches` (batch launches in the traced
run) also the per-launch average of each kernel and of the whole pipeline.
"""
import csv
import glob
import os
import sys


def load(path):
    """Rows {Name, Calls, TotalDurationNs} from a stats CSV or a rocpd database."""
    if os.path.isdir(path):
        found = glob.glob(os.path.join(path, "*kernel_stats.csv"))
        path = found[0] if found else glob.glob(os.path.join(path, "*.db"))[0]
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        q = ("select name, count(*), sum(duration) from kernels group by name "
             "order by sum(duration) desc")
        return [{"Name": n, "Calls": str(c), "TotalDurationNs": str(t), "AverageNs": str(t / c)}
                for n, c, t in con.execute(q)]
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    rows = load(sys.argv[1])
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    total = sum(float(r["TotalDurationNs"]) for r in rows if "k_synth" not in r["Name"])
    print("%-64s %6s %12s %10s %7s" % ("kernel", "calls", "total_us", "avg_us", "share"))
    for r in rows:
        t = float(r["TotalDurationNs"])
        share = 0.0 if "k_synth" in r["Name"] else 100.0 * t / total
        print("%-64s %6s %12.1f %10.1f %6.1f%%" % (r["Name"][:64], r["Calls"], t / 1e3,
                                                  float(r["AverageNs"]) / 1e3, share))
    if launches:
        print("pipeline kernels per batch launch: %.3f ms (input generation excluded)"
              % (total / 1e6 / launches))


if __name__ == "__main__":
    main()
