#!/bin/bash
# Rotate kernel check: deskew/pipeline parity tests, isolated rotate launches
# of 64 A4 sheets (bench --probe), then the default bench.
# usage: tools/rot_probe.sh TAG [UPHIP_ROT_TILES values for the diag build...]
set -o pipefail
tag=${1:-x}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_pipeline_gpu.py tests/test_ops_gpu.py -m gpu -x -q \
  -k "deskew or rotate or a4 or default or c4" --timeout 240 --timeout-method thread > gpurun_out/rt_$tag.log 2>&1 \
  || { tail -30 gpurun_out/rt_$tag.log; exit 1; }
tail -1 gpurun_out/rt_$tag.log
Q="--no-cpu --no-host-io --no-latency"
timeout -k 10 200 python3 bench.py $Q --pages 256 --steps 1 --probe 5 > gpurun_out/rp_$tag.json 2>&1 || { tail gpurun_out/rp_$tag.json; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/rp_$tag.json').read().strip().splitlines()[-1]); print('isolated rotate ms', d['roofline']['avg_launch_ms'], 'verified', d['verified'], d['mismatches'])"
for k in "$@"; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_ROT_TILES=$k timeout -k 10 200 python3 bench.py $Q --tuning --pages 256 --steps 1 --probe 5 > gpurun_out/rpk_$k.json 2>&1 || { tail gpurun_out/rpk_$k.json; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rpk_$k.json').read().strip().splitlines()[-1]); print('tiles/block $k: rotate ms', d['roofline']['avg_launch_ms'], 'mismatches', d['mismatches'])"
done
timeout -k 10 300 python3 bench.py $Q --stages > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { tail gpurun_out/b_$tag.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_$tag.json')); print('bench', d['value'], 'pages/s', d['ms_per_step'], 'ms/step verified', d['verified'], d['mismatches'])"
grep -E "deskew_rotate" gpurun_out/b_$tag.err
