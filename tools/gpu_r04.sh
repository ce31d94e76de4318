#!/bin/bash
# Round-4 GPU round trip: new tests, smoke, the GPU suite, the default bench.
# usage: tools/gpu_r04.sh TAG [pytest -k expr for the first leg]
set -o pipefail
tag=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$2" \
    > gpurun_out/new_$tag.log 2>&1 || { tail -40 gpurun_out/new_$tag.log; exit 1; }
  tail -3 gpurun_out/new_$tag.log
fi
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 \
  || { tail -30 gpurun_out/smoke_$tag.log; exit 1; }
cat gpurun_out/smoke_$tag.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/gt_$tag.log 2>&1 || { tail -30 gpurun_out/gt_$tag.log; exit 1; }
tail -2 gpurun_out/gt_$tag.log
timeout -k 10 300 python3 bench.py --no-cpu --stages > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err \
  || { tail -20 gpurun_out/b_$tag.err; exit 1; }
cat gpurun_out/b_$tag.json; tail -40 gpurun_out/b_$tag.err
