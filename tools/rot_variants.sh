#!/bin/bash
# Isolated k_rotate_cubic_g8f launch (64 sheets, bench.py --probe 5) for
# timing-only variants of the tuning build (make lib DIAG=1; results are
# wrong for all but 0 and 2048): 0 full; 512 arithmetic skipped (all rows
# white); 1536 staging skipped too; 2048 no white-row skip; 4096 no column-sum
# epilogue; 8192 no output stores (combine bits; VARIANTS="..." picks).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-0 512 1536 2048 4096}; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_DOUBLE=$v timeout -k 10 120 \
    python3 bench.py --tuning --no-cpu --no-c4 --no-host-io --no-latency --no-verify --pages 256 \
    --steps 1 --probe 5 > gpurun_out/rv$v.json 2> gpurun_out/rv$v.err || { tail -5 gpurun_out/rv$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rv$v.json').read().strip().splitlines()[-1]); print('variant $v rotate ms', d['roofline']['avg_launch_ms'])"
done
