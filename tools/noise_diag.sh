#!/bin/bash
# noisefilter resolve phases (tuning build): sort / component replay ticks per sheet
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=8 timeout -k 10 200 python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 64 --streams 1 --steps 1 --warmup 0 --no-c4 > gpurun_out/nd.log 2>&1 || { tail gpurun_out/nd.log; exit 1; }
grep "uphip noise: sheet .* n " gpurun_out/nd.log | head -12
