#!/bin/bash
# HBM bytes of the C4 bilinear rotate (k_rotate_lin<F_RGB24>): separate
# FETCH_SIZE and WRITE_SIZE passes over one 4-sheet C4 batch (no single-sheet
# latency runs, so exactly 4 sheets are rotated).  Writes gpurun_out/tc4/c4.json;
# merge it into profiles/traffic.json with
#   python3 profiles/traffic.py --merge-c4 gpurun_out/tc4/c4.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/tc4; rm -rf $out; mkdir -p $out
Q="--config c4 --pages 4 --steps 1 --warmup 0 --no-verify --no-latency --streams 1"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'rotate_lin' --output-format csv -d $out/$c -- python3 bench.py $Q > $out/$c.log 2>&1 || { tail -5 $out/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, json
W, H, SHEETS = 9920, 7016, 4
acc = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/tc4/{c}/**/*counter_collection.csv", recursive=True)[0]
    tot, n = 0.0, 0
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != c:
            continue
        tot += float(r["Counter_Value"]) * 1024
        n += 1
    acc[c] = (tot, n)
    print(c, "dispatches", n, "sheets", SHEETS, "bytes", tot)
fb, nf = acc["FETCH_SIZE"]
wb, nw = acc["WRITE_SIZE"]
doc = {"kernel": "k_rotate_lin<F_RGB24>",
       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                 "--kernel-include-regex rotate_lin -- python3 bench.py --config c4 --pages 4 "
                 "--steps 1 --warmup 0 --no-verify --no-latency --streams 1 (tools/traffic_c4.sh)",
       "dispatches": nf, "sheets": SHEETS,
       "fetch_raw_bytes_per_sheet": int(fb / SHEETS), "write_bytes_per_sheet": int(wb / SHEETS),
       "hbm_bytes_per_sheet": int(2 * fb / SHEETS + wb / SHEETS), "alg_bytes_per_sheet": 2 * W * H * 3}
doc["traffic_over_alg"] = round(doc["hbm_bytes_per_sheet"] / doc["alg_bytes_per_sheet"], 4)
json.dump(doc, open("gpurun_out/tc4/c4.json", "w"), indent=1)
print(json.dumps(doc))
PY
