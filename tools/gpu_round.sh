#!/bin/bash
# One GPU round trip: the GPU test suite, then the default bench (+ stages).
# usage: tools/gpu_round.sh TAG
set -o pipefail
tag=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gt_$tag.log 2>&1 || { tail -30 gpurun_out/gt_$tag.log; exit 1; }
tail -2 gpurun_out/gt_$tag.log
timeout -k 10 240 python3 bench.py --no-cpu --stages > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err || { cat gpurun_out/b_$tag.err | tail; exit 1; }
cat gpurun_out/b_$tag.json gpurun_out/b_$tag.err
