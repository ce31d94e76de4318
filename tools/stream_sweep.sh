#!/bin/bash
# default bench under a few batch x stream shapes (no CPU/host legs)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "64 16" "64 12" "64 20" "80 12" "48 20" "64 16"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --probe 0 --steps 6 --batch $1 --streams $2 > gpurun_out/ss_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ss_$1_$2.json').read().strip().splitlines()[-1]); print('batch $1 streams $2', d['value'])"
done
