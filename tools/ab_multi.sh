#!/bin/bash
# A/B of several builds ab/<name>.so (first name = baseline): rotate/pipeline
# parity tests of every non-baseline build, isolated rotate probe of each,
# then the default-load bench, round-robin, REPS times.
# usage: tools/ab_multi.sh REPS old new c ...
set -o pipefail
reps=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "${@:2}"; do
  cp ab/$v.so unpaper-gpu_amd/lib/libunpaper_hip.so
  timeout -k 10 400 python3 -u -m pytest tests/test_pipeline_gpu.py tests/test_ops_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/abm_tests_$v.log 2>&1 || { tail -30 gpurun_out/abm_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/abm_tests_$v.log)"
done
for v in "$@"; do
  cp ab/$v.so unpaper-gpu_amd/lib/libunpaper_hip.so
  timeout -k 10 120 python3 bench.py --no-cpu --no-host-io --no-latency --pages 256 --steps 1 --probe 5 \
    > gpurun_out/abm_probe_$v.json 2>&1 || { tail gpurun_out/abm_probe_$v.json; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abm_probe_$v.json').read().strip().splitlines()[-1]); print('$v isolated rotate ms', d['roofline']['avg_launch_ms'])"
done
for rep in $(seq "$reps"); do
  for v in "$@"; do
    cp ab/$v.so unpaper-gpu_amd/lib/libunpaper_hip.so
    timeout -k 10 200 python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --probe 0 --steps 6 > gpurun_out/abm_$v.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/abm_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'])"
  done
done
cp ab/$1.so unpaper-gpu_amd/lib/libunpaper_hip.so
