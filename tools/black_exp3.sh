#!/bin/bash
# tuning experiment on the C4 replay: UPHIP_DIAG_NOISE=16|$1 (32: no image stores)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 16 $((16|$1)); do
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=$v timeout -k 10 200 python3 bench.py --config c4 --tuning --steps 1 --warmup 0 --no-verify > gpurun_out/bx4_$v.log 2>&1 || { tail gpurun_out/bx4_$v.log; exit 1; }
echo "== $v"; grep "uphip black" gpurun_out/bx4_$v.log | sort -t' ' -k6 -n | tail -1
done
