#!/bin/bash
# Quick GPU check: pipeline parity tests, isolated rotate probe, default bench.
# usage: tools/gpu_quick.sh TAG
set -o pipefail
tag=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gq_$tag.log 2>&1 || { tail -30 gpurun_out/gq_$tag.log; exit 1; }
tail -1 gpurun_out/gq_$tag.log
timeout -k 10 120 python3 bench.py --no-cpu --pages 256 --steps 1 --probe 5 > gpurun_out/rp_$tag.json 2>&1 || { tail gpurun_out/rp_$tag.json; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/rp_$tag.json').read().strip().splitlines()[-1]); print('isolated rotate ms', d['roofline']['avg_launch_ms'])"
timeout -k 10 240 python3 bench.py --no-cpu --stages > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { tail gpurun_out/b_$tag.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_$tag.json')); print('bench', d['value'], 'pages/s', d['ms_per_step'], 'ms/step')"
cat gpurun_out/b_$tag.err
