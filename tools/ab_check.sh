#!/bin/bash
# Parity of the new build (pipeline + rotate op tests), isolated rotate probe
# of both builds, then the load A/B of tools/ab_lib.sh.  ab/old.so, ab/new.so
# prepared as tools/ab_lib.sh describes.
set -o pipefail
reps=${1:-3}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cp ab/new.so unpaper-gpu_amd/lib/libunpaper_hip.so
timeout -k 10 400 python3 -u -m pytest tests/test_pipeline_gpu.py tests/test_ops_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/abc_tests.log 2>&1 || { tail -30 gpurun_out/abc_tests.log; exit 1; }
tail -1 gpurun_out/abc_tests.log
for v in old new; do
  cp ab/$v.so unpaper-gpu_amd/lib/libunpaper_hip.so
  timeout -k 10 120 python3 bench.py --no-cpu --no-host-io --no-latency --pages 256 --steps 1 --probe 5 \
    > gpurun_out/abc_probe_$v.json 2>&1 || { tail gpurun_out/abc_probe_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abc_probe_$v.json').read().strip().splitlines()[-1]); print('$v isolated rotate ms', d['roofline']['avg_launch_ms'])"
done
bash tools/ab_lib.sh "$reps"
