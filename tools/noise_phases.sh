#!/bin/bash
# k_noise_classify phase costs: the tuning build's early exits (UPHIP_DIAG_NOISE
# 1: after the region rows, 2: after the large-component pass, 3: after the
# candidate list), one-stream kernel time per 64-sheet launch under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/np
for v in 0 1 2 3; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=$v timeout -s KILL 120 \
    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/np/n$v -- python3 bench.py --tuning \
    --no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0 \
    > gpurun_out/np/n$v.log 2>&1 || { tail -5 gpurun_out/np/n$v.log; exit 1; }
  echo "UPHIP_DIAG_NOISE=$v: $(python3 profiles/summarize.py gpurun_out/np/n$v 2 | grep k_noise_classify)"
done
