#!/bin/bash
# blackfilter tests, then FETCH / WRITE passes over two C3 batches: per-kernel MB/page
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/btr; rm -rf $out; mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "black or c4 or bench or flood" > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
Q="--no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $out/$c -- python3 bench.py $Q > $out/$c.log 2>&1 || { tail -5 $out/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
def per(c):
    acc = collections.defaultdict(float)
    f = glob.glob(f"gpurun_out/btr/{c}/**/*counter_collection.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == c: acc[r["Kernel_Name"].split("(")[0]] += float(r["Counter_Value"]) * 1024
    return acc
F, W = per("FETCH_SIZE"), per("WRITE_SIZE")
tot = 0
for k in sorted(set(F) | set(W)):
    if "synth" in k: continue
    f, w = 2 * F.get(k, 0) / 128 / 1e6, W.get(k, 0) / 128 / 1e6
    tot += f + w
    if "black" in k: print(f"{k[:40]:40s} fetch2 {f:6.2f} write {w:6.2f} MB/page")
print("pipeline total %.2f MB/page" % tot)
PY
