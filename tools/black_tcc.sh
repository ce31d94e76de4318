#!/bin/bash
# L2 counters of k_black_resolve on the C4 workload
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/btcc; rm -rf $out; mkdir -p $out
Q="--config c4 --tuning --steps 1 --warmup 0 --no-verify"
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_ATOMIC_sum --kernel-trace --output-format csv -d $out/p1 -- python3 bench.py $Q > $out/p1.log 2>&1 || { tail -3 $out/p1.log; }
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_PENDING_STALL_CYCLES_sum --kernel-trace --output-format csv -d $out/p2 -- python3 bench.py $Q > $out/p2.log 2>&1 || { tail -3 $out/p2.log; }
python3 - <<'PY'
import csv, glob, collections
for tag in ("p1", "p2"):
    acc = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/btcc/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_black_resolve" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(acc.items()): print(tag, k, v)
PY
