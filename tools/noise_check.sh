#!/bin/bash
# noisefilter parity tests, the resolve phases (tuning build), and kernel durations
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${1:-noise or golden or A1 or C1 or E1 or bench_configuration}" > gpurun_out/noise_t.log 2>&1 || { tail -30 gpurun_out/noise_t.log; exit 1; }
tail -1 gpurun_out/noise_t.log
bash tools/noise_diag.sh | head -4
bash tools/blur_prof.sh | grep noise_resolve
