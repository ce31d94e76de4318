#!/bin/bash
# blackfilter replay: black/C4/bench-hash GPU tests, then the replay counters
# (tuning build) on the C4 sheets
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${1:-black or c4 or flood}" > gpurun_out/blk_t.log 2>&1 || { tail -30 gpurun_out/blk_t.log; exit 1; }
tail -1 gpurun_out/blk_t.log
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --config c4 --tuning --steps 1 --warmup 0 --no-verify > gpurun_out/bc4.log 2>&1 || { tail gpurun_out/bc4.log; exit 1; }
grep "uphip black" gpurun_out/bc4.log | sort -t' ' -k6 -n | tail -3
