#!/bin/bash
# Isolated rotate time for several tiles-per-block settings (UPHIP_ROT_PER_BLOCK).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 200 python3 -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "default or deskew or sizes" > gpurun_out/pb_tests.log 2>&1 || { tail -20 gpurun_out/pb_tests.log; exit 1; }
tail -1 gpurun_out/pb_tests.log
for v in 1 2 4 8; do
  UPHIP_ROT_PER_BLOCK=$v timeout -k 10 120 python3 bench.py --no-cpu --pages 256 --steps 1 --probe 5 > gpurun_out/pb$v.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/pb$v.json').read().strip().splitlines()[-1]); print('per_block $v rotate ms', d['roofline']['avg_launch_ms'])"
done
