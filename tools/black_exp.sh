#!/bin/bash
# tuning experiment: replay counters with UPHIP_DIAG_NOISE=$1 (bit 16 print, bit 32 no image stores)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=$v timeout -k 10 200 python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 4 --batch 4 --streams 1 --steps 1 --warmup 0 > gpurun_out/bx_$v.log 2>&1 || { tail gpurun_out/bx_$v.log; exit 1; }
echo "== $v"; grep "uphip black" gpurun_out/bx_$v.log | head -20
done
