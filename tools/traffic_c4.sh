#!/bin/bash
# HBM bytes of the C4 bilinear rotate (k_rotate_lin<F_RGB24>): separate
# FETCH_SIZE and WRITE_SIZE passes over one 4-sheet C4 run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/tc4; rm -rf $out; mkdir -p $out
Q="--config c4 --pages 4 --steps 1 --warmup 0 --no-verify --streams 1"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'rotate_lin' --output-format csv -d $out/$c -- python3 bench.py $Q > $out/$c.log 2>&1 || { tail -5 $out/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, json
W, H = 9920, 7016
acc = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/tc4/{c}/**/*counter_collection.csv", recursive=True)[0]
    tot, sheets, n = 0.0, 0.0, 0
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != c:
            continue
        tot += float(r["Counter_Value"]) * 1024
        n += 1
    # sheets rotated: the 4-sheet batch and bench.py's 4 single-sheet latency
    # runs (run_c4); a sheet whose mask 1 depends on deskew 0 takes two launches
    sheets = 4 + 4
    acc[c] = (tot, sheets, n)
    print(c, "dispatches", n, "sheets", sheets, "bytes", tot)
fb, fs, _ = acc["FETCH_SIZE"]
wb, ws, _ = acc["WRITE_SIZE"]
doc = {"kernel": "k_rotate_lin<F_RGB24>",
       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                 "--kernel-include-regex rotate_lin -- python3 bench.py --config c4 --pages 4 "
                 "--steps 1 --warmup 0 --no-verify --streams 1 (tools/traffic_c4.sh)",
       "fetch_raw_bytes_per_sheet": int(fb / fs), "write_bytes_per_sheet": int(wb / ws),
       "hbm_bytes_per_sheet": int(2 * fb / fs + wb / ws), "alg_bytes_per_sheet": 2 * W * H * 3}
json.dump(doc, open("gpurun_out/tc4/c4.json", "w"), indent=1)
print(json.dumps(doc))
PY
