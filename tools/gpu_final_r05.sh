#!/bin/bash
# Round-5 evidence on one GPU, each step under its own limit (gpurun_out/r05f/):
# the full GPU suite, smoke(), the default bench line, the JPEG, JPEG 2000
# and PDF runner lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05f
mkdir -p $o
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $o/gpu_tests.log 2>&1 || { tail -40 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 400 python3 bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail -20 $o/bench_default.err; exit 1; }
tail -c 600 $o/bench_default.json
timeout -k 10 300 python3 bench.py --config jpeg --pages 1024 > $o/bench_jpeg.json 2> $o/bench_jpeg.err || { tail -20 $o/bench_jpeg.err; exit 1; }
timeout -k 10 300 python3 bench.py --config jp2 --pages 512 > $o/bench_jp2.json 2> $o/bench_jp2.err || { tail -20 $o/bench_jp2.err; exit 1; }
timeout -k 10 300 python3 bench.py --config pdf > $o/bench_pdf.json 2> $o/bench_pdf.err || { tail -20 $o/bench_pdf.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench_jpeg", "bench_jp2", "bench_pdf"):
    d = json.loads(open("gpurun_out/r05f/%s.json" % n).read().strip().splitlines()[-1])
    print(n, d["value"], d["unit"], "verified", d.get("verified"))
PY
