#!/bin/bash
# blur parity tests, then the blur/noise kernels' launch durations
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${1:-blur or golden or A1 or C1 or E1 or bench_configuration}" > gpurun_out/blur_t.log 2>&1 || { tail -30 gpurun_out/blur_t.log; exit 1; }
tail -1 gpurun_out/blur_t.log
bash tools/blur_prof.sh
