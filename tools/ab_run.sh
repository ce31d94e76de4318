#!/bin/bash
# parity of the filter/pipeline suites with the new library, then an A/B of the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cp ab/new.so unpaper-gpu_amd/lib/libunpaper_hip.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filters_gpu.py tests/test_pipeline_gpu.py tests/test_ops_gpu.py > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bash tools/ab_lib.sh ${1:-3}
