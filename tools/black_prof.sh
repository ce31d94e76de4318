#!/bin/bash
# k_black_resolve launch durations (production build, no timers): C4 (16
# sheets, 4 per launch) and one 64-page C3 batch, under rocprofv3 kernel-trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/bprof; rm -rf $out; mkdir -p $out
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $out/c4 -- python3 bench.py --config c4 --tuning --steps 1 --warmup 0 --no-verify > $out/c4.log 2>&1 || { tail $out/c4.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $out/c3 -- python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 64 --streams 1 --steps 1 --warmup 0 --no-c4 > $out/c3.log 2>&1 || { tail $out/c3.log; exit 1; }
python3 - <<'PY'
import csv, glob
for tag in ("c4", "c3"):
    rows = []
    for f in glob.glob(f"gpurun_out/bprof/{tag}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    for key in ("k_black_resolve", "k_black_planes", "k_black_paint", "k_black_cand"):
        d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if key in r["Kernel_Name"])
        if d: print(f"{tag} {key:16s} n={len(d):3d} sum={sum(d):9.1f} us max={d[-1]:9.1f} med={d[len(d)//2]:8.1f}")
PY
