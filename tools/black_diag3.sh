#!/bin/bash
# replay counters (tuning build) on the C4 workload and one C3 batch
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --config c4 --tuning --steps 1 --warmup 0 --no-verify > gpurun_out/bc4.log 2>&1 || { tail gpurun_out/bc4.log; exit 1; }
grep "uphip black" gpurun_out/bc4.log | sort -t' ' -k6 -n | tail -2
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 64 --streams 1 --steps 1 --warmup 0 --no-c4 > gpurun_out/bc3.log 2>&1 || { tail gpurun_out/bc3.log; exit 1; }
grep -c "uphip black" gpurun_out/bc3.log; grep "uphip black" gpurun_out/bc3.log | head -2
