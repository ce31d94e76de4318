#!/bin/bash
# Marginal cost of kernels in the 16-stream steady state: the tuning build
# launches a kernel twice when its UPHIP_DIAG_DOUBLE bit is set
# (UPH_LAUNCH_DIAG); the drop in pages/s against 0 is what the kernel costs the
# pipeline.  Bits: 1 rotation band, 16 rotation points, 128 rotation final +
# line walk, 2 rotate, 4 moves, 8 copy, 32 gray cells, 64 blur counts,
# 131072 noise classify, 262144 GRAY8 decode.  usage: BITS="0 1 16 128" tools/ab_double.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${BITS:-0 1 16 128 2}; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_DOUBLE=$v timeout -k 10 200 \
    python3 bench.py --tuning --no-cpu --no-c4 --no-host-io --no-latency --no-verify --probe 0 \
    > gpurun_out/ad$v.json 2> gpurun_out/ad$v.err || { tail -5 gpurun_out/ad$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ad$v.json').read().strip().splitlines()[-1]); print('double $v pages/s', d['value'])"
done
