#!/bin/bash
# blackfilter replay (round 5): the black/C4/flood/bench-hash GPU tests, then
# the C4 leg (the heaviest band sheet's blackfilter stage) and the C3 leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05; mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${K:-black or c4 or flood or bench}" > $o/blk_t.log 2>&1 || { tail -30 $o/blk_t.log; exit 1; }
tail -1 $o/blk_t.log
timeout -k 10 400 python3 bench.py --config c4 > $o/blk_c4.json 2> $o/blk_c4.err || { tail $o/blk_c4.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05/blk_c4.json").read().strip().splitlines()[-1])
print("c4 sheets/s", d["value"], "verified", d["verified"], "latency", d["latency_ms"], "band", d["latency_band_ms"],
      "band blackfilter", d["latency_band_stages_ms"]["blackfilter"], "per sheet", d["latency_per_sheet_ms"])
PY
