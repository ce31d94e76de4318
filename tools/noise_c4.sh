#!/bin/bash
# noise/C4 parity tests, then the C4 line (latency and its noisefilter stage)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "noise or c4 or golden or C1 or rgb" > gpurun_out/nc4_t.log 2>&1 || { tail -30 gpurun_out/nc4_t.log; exit 1; }
tail -1 gpurun_out/nc4_t.log
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/c4b.json 2> gpurun_out/c4b.err || { tail gpurun_out/c4b.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/c4b.json').read().strip().splitlines()[-1])
print('C4', d['value'], d['verified'], d['mismatches'], 'latency', d['latency_ms'], d['latency_stages_ms']['noisefilter'])"
