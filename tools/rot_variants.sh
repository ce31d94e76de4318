#!/bin/bash
# Isolated rotate-kernel time for timing-only variants (results are wrong for
# 512/1024): 256 old kernel, 512 skip compute, 1024 skip staging, 2048 no white skip.
set -o pipefail
for v in 0 512 1536 2048; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_DOUBLE=$v timeout -k 10 120 python3 bench.py --no-cpu --pages 256 --steps 1 --probe 5 > gpurun_out/rv$v.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/rv$v.json').read().strip().splitlines()[-1]); print('variant $v rotate ms', d['roofline']['avg_launch_ms'])"
done
