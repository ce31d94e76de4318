#!/bin/bash
# Round evidence: the full GPU suite, the default bench line, the C4 mode.
set -o pipefail
tag=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/full_$tag.log 2>&1 || { tail -40 gpurun_out/full_$tag.log; exit 1; }
tail -3 gpurun_out/full_$tag.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
  || { tail -30 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
timeout -k 10 200 python3 bench.py --config c4 --steps 3 > gpurun_out/c4_$tag.json 2> gpurun_out/c4_$tag.err \
  || { tail -30 gpurun_out/c4_$tag.err; exit 1; }
cat gpurun_out/c4_$tag.json
