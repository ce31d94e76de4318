#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory.

usage: summarize.py <rocprofv3 output dir or *_kernel_stats.csv> [launches]
                    [--last KERNEL K [--per-stage N]]

Prints kernels by total time; with `launches` (batch launches in the traced
run) also the per-launch average of each kernel and of the whole pipeline.
With --last, also the average duration of the last K dispatches of KERNEL
from the per-dispatch trace (*kernel_trace.csv): bench.py's isolated probe
launches of the roofline kernel run after everything else, so this is the
rocprof figure to set next to bench.py's `roofline.avg_launch_ms`.
"""
import csv
import glob
import os
import sys


def load(path):
    """Rows {Name, Calls, TotalDurationNs} from a stats CSV or a rocpd database."""
    if os.path.isdir(path):
        found = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
        path = found[0] if found else glob.glob(os.path.join(path, "**", "*.db"),
                                                recursive=True)[0]
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        q = ("select name, count(*), sum(duration) from kernels group by name "
             "order by sum(duration) desc")
        return [{"Name": n, "Calls": str(c), "TotalDurationNs": str(t), "AverageNs": str(t / c)}
                for n, c, t in con.execute(q)]
    with open(path) as f:
        return list(csv.DictReader(f))


def last_dispatches(path, kernel, k):
    """Durations (us) of the last k dispatches of `kernel` in start order."""
    found = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not found:
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        if not dbs:
            return []
        import sqlite3
        con = sqlite3.connect(dbs[0])
        rows = con.execute("select start, end from kernels where name like ? order by start",
                           ("%" + kernel + "%",)).fetchall()
        return [(e - s) / 1e3 for s, e in rows[-k:]]
    with open(found[0]) as f:
        rows = [r for r in csv.DictReader(f) if kernel in r.get("Kernel_Name", "")]
    # full-batch launches only: bench.py's single-page latency runs (grid z =
    # 1) come after its probes
    zmax = max((int(r.get("Grid_Size_Z", 1)) for r in rows), default=1)
    rows = [r for r in rows if int(r.get("Grid_Size_Z", 1)) == zmax]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[-k:]]


def main():
    argv = sys.argv[1:]
    last = None
    if "--last" in argv:
        i = argv.index("--last")
        last = (argv[i + 1], int(argv[i + 2]))
        del argv[i:i + 3]
    rows = load(argv[0])
    launches = int(argv[1]) if len(argv) > 1 else 0
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
    per = 1  # dispatches per stage: the GRAY8 bicubic rotation is two launches
    if "--per-stage" in argv:  # (sheets split by window size), summed per stage
        per = int(argv[argv.index("--per-stage") + 1])
    if last and os.path.isdir(argv[0]):
        d = last_dispatches(argv[0], last[0], last[1] * per)
        if per > 1 and d:
            print("last %d dispatches of %s: %s us" % (len(d), last[0], " ".join("%.1f" % v for v in d)))
            d = [sum(d[i:i + per]) for i in range(0, len(d) - per + 1, per)]
            last = ("%s (stage = %d launches)" % (last[0], per), last[1])
        if d:
            print("last %d dispatches of %s: %s us, average %.1f us"
                  % (len(d), last[0], " ".join("%.1f" % v for v in d), sum(d) / len(d)))


if __name__ == "__main__":
    main()
