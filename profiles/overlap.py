#!/usr/bin/env python3
"""Concurrency of a rocprofv3 --kernel-trace run: union of busy time, summed
kernel time, and the share of time each kernel family runs alone or
overlapped.  usage: overlap.py <trace dir> [t0_frac t1_frac]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
ev = []
for r in csv.DictReader(open(kt)):
    n = r["Kernel_Name"]
    if "synth" in n or "rocclr" in n:
        continue
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0].replace("void ", "")[:40]))
ev.sort()
t0 = min(e[0] for e in ev)
t1 = max(e[1] for e in ev)
if len(sys.argv) > 3:
    a, b = float(sys.argv[2]), float(sys.argv[3])
    t0, t1 = t0 + a * (t1 - t0), t0 + b * (t1 - t0)
    ev = [e for e in ev if e[1] > t0 and e[0] < t1]
# sweep
pts = []
for s, e, n in ev:
    pts.append((max(s, t0), 1, n))
    pts.append((min(e, t1), -1, n))
pts.sort()
active = collections.Counter()
last = t0
busy = 0.0
conc = collections.Counter()   # time by number of concurrent kernels
alone = collections.Counter()  # time a family runs with nothing else
share = collections.Counter()  # time-weighted share (1/n per active kernel)
for t, dlt, n in pts:
    dt = t - last
    k = sum(active.values())
    if dt > 0 and k:
        busy += dt
        conc[min(k, 8)] += dt
        for name, c in active.items():
            if c:
                share[name] += dt * c / k
        if k == 1:
            alone[next(n_ for n_, c in active.items() if c)] += dt
    active[n] += dlt
    last = t
span = t1 - t0
summ = sum(min(e, t1) - max(s, t0) for s, e, _ in ev)
print("span %.2f ms, busy %.2f ms (%.1f%%), summed kernel time %.2f ms (x%.2f)" %
      (span / 1e6, busy / 1e6, 100 * busy / span, summ / 1e6, summ / max(busy, 1)))
print("time by concurrency:", {k: round(v / span * 100, 1) for k, v in sorted(conc.items())})
print("%-40s %9s %9s" % ("kernel", "share_ms", "alone_ms"))
for n, v in share.most_common(20):
    print("%-40s %9.2f %9.2f" % (n, v / 1e6, alone[n] / 1e6))
