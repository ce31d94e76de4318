#!/bin/bash
# A/B of two builds of libunpaper_hip.so under the default bench load, on the
# GPU box.  Prepare in the build container:
#   mkdir -p ab && cp unpaper-gpu_amd/lib/libunpaper_hip.so ab/new.so
#   git stash && make lib && cp unpaper-gpu_amd/lib/libunpaper_hip.so ab/old.so && git stash pop
# then: gpurun -- 'bash tools/ab_lib.sh [reps]'   (ab/ is scratch: delete it after)
set -o pipefail
reps=${1:-3}
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in $(seq "$reps"); do
  for v in old new; do
    cp ab/$v.so unpaper-gpu_amd/lib/libunpaper_hip.so
    timeout -k 10 200 python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --probe 0 --no-c4 --steps 6 > gpurun_out/ab_$v.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'])"
  done
done
cp ab/new.so unpaper-gpu_amd/lib/libunpaper_hip.so
