#!/bin/bash
# k_noise_classify time with its phases cut off one by one (tuning build,
# UPHIP_DIAG_NOISE=1: after the bit rows, 2: after the candidate lists,
# 3: after the small floods; 0: whole kernel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 0 1 2 3; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=$v timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/np_$v -- \
    python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0 --no-c4 > gpurun_out/np_$v.log 2>&1 || { tail -5 gpurun_out/np_$v.log; exit 1; }
  f=$(find gpurun_out/np_$v -name '*kernel_stats.csv' | head -1)
  echo "diag $v: $(grep noise_classify $f | cut -d, -f2-4)"
done
