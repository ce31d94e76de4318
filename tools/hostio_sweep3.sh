#!/bin/bash
# host-fed figure 2 vs chunk size and stream count
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "32 8" "16 12" "8 16" "8 24" "4 32"; do
  set -- $cfg
  timeout -k 10 150 python3 bench.py --no-cpu --no-latency --no-c4 --probe 0 --steps 2 --warmup 1 --host-batch $1 --host-streams $2 > gpurun_out/hio_$1_$2.json 2>gpurun_out/hio.err || { tail -3 gpurun_out/hio.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/hio_$1_$2.json').read().strip().splitlines()[-1]); h=d['host_io']
print('batch $1 streams $2:', h['h2d_d2h']['value'], 'pages/s; pnm', h['pnm_write']['value'])"
done
