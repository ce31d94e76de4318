#!/bin/bash
# blackfilter replay check: black / C4 / bench-hash GPU tests, replay counters
# (tuning build) on C4 and C3, then the default bench line with C4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${1:-black or c4 or bench or flood}" > gpurun_out/blk_t.log 2>&1 || { tail -30 gpurun_out/blk_t.log; exit 1; }
tail -2 gpurun_out/blk_t.log
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --config c4 --tuning --steps 1 --warmup 0 --no-verify > gpurun_out/bc4.log 2>&1 || { tail gpurun_out/bc4.log; exit 1; }
grep "uphip black" gpurun_out/bc4.log | sort -t' ' -k6 -n | tail -4
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 64 --streams 1 --steps 1 --warmup 0 --no-c4 > gpurun_out/bc3.log 2>&1 || { tail gpurun_out/bc3.log; exit 1; }
grep -c "uphip black" gpurun_out/bc3.log; grep "uphip black" gpurun_out/bc3.log | head -3
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_blk.json 2> gpurun_out/bench_blk.err || { tail gpurun_out/bench_blk.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_blk.json').read().strip().splitlines()[-1]); c=d.get('c4',{})
print('C3', d['value'], d.get('verified'), d.get('mismatches'), 'C4', c.get('value'), c.get('verified'), c.get('mismatches'), c.get('stages_ms_per_step'))"
