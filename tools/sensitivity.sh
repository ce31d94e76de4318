#!/bin/bash
# Marginal cost of idempotent kernels under the multi-stream bench load:
# each UPHIP_DIAG_DOUBLE bit launches one kernel twice (common.h).
set -o pipefail
out=${1:-gpurun_out/sens}
mkdir -p "$out"
for b in 0 1 2 4 8 32 64 128; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_DOUBLE=$b timeout -k 10 120 python3 bench.py --no-cpu --probe 0 --steps 5 \
    > "$out/d$b.json" 2> "$out/d$b.err" || exit 1
  python3 -c "import json; d=json.load(open('$out/d$b.json')); print('double $b', d['ms_per_step'], d['value'])"
done
