#!/bin/bash
# counters of k_black_resolve on one C3 batch: instruction mix, waits, icache
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/bpmc; rm -rf $out; mkdir -p $out


Q="${BQ:---tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 64 --streams 1 --steps 1 --warmup 0 --no-c4}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_LDS --kernel-trace --output-format csv -d $out/p1 -- python3 bench.py $Q > $out/p1.log 2>&1 || { tail -3 $out/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $out/p2 -- python3 bench.py $Q > $out/p2.log 2>&1 || { tail -3 $out/p2.log; }
python3 - <<'PY'
import csv, glob, collections
for tag in ("p1", "p2"):
    acc = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/bpmc/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_black_resolve" in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(acc.items()): print(tag, k, v)
PY
