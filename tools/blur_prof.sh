#!/bin/bash
# blur kernels' launch durations: one 64-page batch and the C2 single-page runs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/blurprof; rm -rf $out; mkdir -p $out
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $out/t -- python3 bench.py --no-cpu --no-host-io --no-c4 --no-verify --probe 0 --pages 64 --streams 1 --steps 1 --warmup 0 > $out/t.log 2>&1 || { tail $out/t.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
rows = []
for f in glob.glob("gpurun_out/blurprof/t/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if any(t in n for t in (os.environ.get("KPAT", "blur,noise").split(","))):
        g = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        d[(n.split("(")[0][-40:], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    v.sort(); print("%-42s grid %-10s n=%3d med %8.1f us  min %8.1f" % (k[0], k[1], len(v), v[len(v)//2], v[0]))
PY
