#!/bin/bash
# black-resolve replay counters (tuning build) + single-stream stage times of
# the product build; tools/black_run.sh adds the parity tests and an A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 8 --batch 8 --streams 1 --steps 1 --warmup 0 > gpurun_out/bk.log 2>&1 || { tail gpurun_out/bk.log; exit 1; }
grep "uphip black" gpurun_out/bk.log | head -4
timeout -k 10 200 python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --probe 0 --steps 2 --warmup 1 --streams 1 --pages 128 --stages > gpurun_out/stages_new.json 2> gpurun_out/stages_new.txt || exit 1
grep -E "black|noise|rotate" gpurun_out/stages_new.txt
