#!/bin/bash
# JPEG GPU tests, then the JPEG runner bench under rocprofv3 (kernel stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05
mkdir -p $o
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "jpeg" \
  > $o/gpu_tests_jpeg.log 2>&1 || { tail -40 $o/gpu_tests_jpeg.log; exit 1; }
tail -2 $o/gpu_tests_jpeg.log
tools/prof_jpeg.sh
