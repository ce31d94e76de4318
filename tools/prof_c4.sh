#!/bin/bash
# rocprofv3 kernel trace of the C4 workload (and optionally the default bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -- \
  python3 bench.py --config c4 --pages 8 --steps 2 --warmup 1 --no-verify > gpurun_out/prof_c4.log 2>&1 \
  || { tail -20 gpurun_out/prof_c4.log; exit 1; }
f=$(find gpurun_out/prof_c4 -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-60s %6s %10.3f ms %9.3f ms" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"])/1e6, float(r["AverageNs"])/1e6))
PY
