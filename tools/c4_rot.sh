#!/bin/bash
# C4: parity tests, then the C4 bench line's bilinear rotate roofline
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${1:-c4 or linear or lin or bilinear}" > gpurun_out/c4_t.log 2>&1 || { tail -30 gpurun_out/c4_t.log; exit 1; }
tail -1 gpurun_out/c4_t.log
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail gpurun_out/c4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/c4.json').read().strip().splitlines()[-1]); r=d['roofline']
print('C4', d['value'], d.get('verified'), d.get('mismatches'), 'rot ms', r['avg_launch_ms'], 'frac', r['frac'])"
