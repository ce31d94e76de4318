#!/bin/bash
# C4-path check: deskew/C4 GPU tests, then the C4 kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${1:-c4 or deskew or interp or rotate}" > gpurun_out/c4t.log 2>&1 || { tail -30 gpurun_out/c4t.log; exit 1; }
tail -2 gpurun_out/c4t.log
tools/prof_c4.sh
