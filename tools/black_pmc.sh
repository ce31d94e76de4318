#!/bin/bash
# PMC pass over the black replay (8 sheets, one stream, product build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d gpurun_out/pmc_black -- \
  python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 8 --batch 8 --streams 1 --steps 1 --warmup 0 > gpurun_out/pmc_black.log 2>&1 || { tail -5 gpurun_out/pmc_black.log; exit 1; }
f=$(find gpurun_out/pmc_black -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "black_resolve" in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k, {c: int(x) for c, x in sorted(v.items())})
PY
