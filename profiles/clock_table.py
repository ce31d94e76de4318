#!/usr/bin/env python3
"""Per-kernel effective clock (GRBM_GUI_ACTIVE / duration) and VALU issue
fraction (SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x active cycles)) from a
rocprofv3 --kernel-trace --pmc run (tools/pmc_clock.sh).

usage: clock_table.py <run dir> [sheets-per-launch out.json]
With the last two arguments it also writes per-kernel VALU instructions per
sheet and the effective clock, which bench.py reads (--valu) to report the
roofline kernel's VALU-issue fraction next to its HBM fraction."""
import json
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(cc)):
    k = r["Kernel_Name"][:56]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    agg[k]["_n_" + r["Counter_Name"]] += 1
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
dur = collections.defaultdict(float)
if kt:
    for r in csv.DictReader(open(kt[0])):
        dur[r["Kernel_Name"][:56]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
doc = {"source": "rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES "
              "SQ_INSTS_SALU SQ_BUSY_CYCLES (tools/pmc_clock.sh)",
       "formula": "VALU issue fraction = SQ_INSTS_VALU x 4 cycles (wave64 on a 16-lane SIMD) / "
                  "(1024 SIMDs x clock x kernel time)",
       "kernels": {}}
launches = collections.Counter()
if kt:
    for r in csv.DictReader(open(kt[0])):
        launches[r["Kernel_Name"][:56]] += 1
# GRBM_GUI_ACTIVE / 8 / wall time is the effective clock only for long
# dispatches (MI355X_MICROARCH.md, DVFS give-back: it reads high below about
# 0.3 ms and is within 3 % from 10 ms up); a kernel of a few waves keeps the
# GUI busy as long as it runs and reads high too.  A kernel's own figure is
# used only from dispatches of >= 0.5 ms that come out at or below the chip's
# 2.4 GHz; every other kernel gets the median of those ("*" in the table), so
# no clock above 2.4 GHz is reported and no VALU fraction is understated.
LONG_MS, MAX_GHZ = 0.5, 2.4
clk = {}
for k, v in agg.items():
    t = dur.get(k, 0.0)
    n = launches.get(k, 0) or 1
    if t > 0 and t * 1e3 / n >= LONG_MS:
        ghz = v.get("GRBM_GUI_ACTIVE", 0.0) / 8 / t / 1e9
        if 0 < ghz <= MAX_GHZ:
            clk[k] = ghz
long_ghz = min(sorted(clk.values())[len(clk) // 2], MAX_GHZ) if clk else MAX_GHZ
print("%-56s %9s %9s %8s %9s %9s" % ("kernel", "dur_ms", "GHz", "VALU%", "VALU/wave", "SALU/wave"))
for k, v in sorted(agg.items(), key=lambda kv: -dur.get(kv[0], 0)):
    t = dur.get(k, 0.0)
    ghz = clk.get(k, long_ghz)
    gui = ghz * 1e9 * t  # active cycles of the kernel
    valu = v.get("SQ_INSTS_VALU", 0.0)
    frac = valu * 4 / (1024 * gui) if gui > 0 else 0.0
    waves = v.get("SQ_WAVES", 0.0)
    salu = v.get("SQ_INSTS_SALU", 0.0)
    print("%-56s %9.3f %9s %8.1f %9.0f %9.0f" % (k, t * 1e3, ("%.3f" % ghz) + ("" if k in clk else "*"),
                                                100 * frac, valu / waves if waves else 0,
                                                salu / waves if waves else 0))
    n = launches.get(k, 0)
    if len(sys.argv) > 3 and n:
        doc["kernels"][k.split("(")[0].split("::")[-1].split("<")[0] + ("<" + k.split("<")[1].split(">")[0] + ">" if "<" in k else "")] = {
            "launches": n, "ms_per_launch": round(t * 1e3 / n, 4), "clock_ghz": round(ghz, 3),
            "clock_from": "GRBM_GUI_ACTIVE" if k in clk else "assumed: median of the run's measured kernels",
            "valu_insts_per_sheet": int(valu / n / int(sys.argv[2])), "valu_issue_frac": round(frac, 4),
            "valu_insts_per_wave": round(valu / waves, 1) if waves else None,
            "salu_insts_per_wave": round(salu / waves, 1) if waves else None}
print("* clock assumed: the median (%.3f GHz) of the kernels measured at >= %.1f ms a launch and <= %.1f GHz"
      % (long_ghz, LONG_MS, MAX_GHZ))
if len(sys.argv) > 3:
    with open(sys.argv[3], "w") as f:
        json.dump(doc, f, indent=1)
