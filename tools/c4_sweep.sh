#!/bin/bash
# C4 throughput vs sheets per batch (streams = sheets / batch, up to 16)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 1 2 4; do
  timeout -k 10 200 python3 bench.py --config c4 --steps 3 --batch $b --no-verify > gpurun_out/c4s_$b.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/c4s_$b.json').read().strip().splitlines()[-1]); print('batch $b', d['value'], d['config'], d['stages_ms_per_step']['blackfilter'])"
done
