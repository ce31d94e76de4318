#!/bin/bash
# SQ counters of the linear rotate on C4 (4 sheets + the latency runs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
Q="--config c4 --pages 4 --steps 1 --warmup 0 --no-verify --streams 1"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'rotate_lin' --output-format csv -d gpurun_out/pmcrl -- python3 bench.py $Q > gpurun_out/pmcrl.log 2>&1 || { tail -5 gpurun_out/pmcrl.log; exit 1; }
python3 - "$(find gpurun_out/pmcrl -name '*counter_collection.csv' | head -1)" <<'PY'
import csv, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    key = (r["Dispatch_Id"], r["Grid_Size"] if "Grid_Size" in r else "")
    d[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(d.items(), key=lambda kv: int(kv[0][0])):
    n = max(v.get("SQ_WAVES", 1), 1)
    print(k, int(n), " ".join("%s=%.0f" % (c[3:], v[c] / n) for c in sorted(v) if c != "SQ_WAVES"))
PY
