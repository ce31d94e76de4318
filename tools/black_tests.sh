#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filters_gpu.py -k black > gpurun_out/black_t.log 2>&1; tail -30 gpurun_out/black_t.log
