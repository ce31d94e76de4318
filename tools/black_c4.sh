#!/bin/bash
# black replay counters on the C4 workload (tuning build)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --config c4 --tuning --steps 1 --warmup 0 --no-verify > gpurun_out/bc4.log 2>&1 || { tail gpurun_out/bc4.log; exit 1; }
grep "uphip black" gpurun_out/bc4.log | head -8
