#!/bin/bash
# GPU check of a working tree: selected test files, then the default bench.
# usage: tools/gpu_check.sh TAG "tests/test_a.py tests/test_b.py" [bench args...]
set -o pipefail
tag=${1:-x}; tests=${2:-tests}; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest $tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -3 gpurun_out/t_$tag.log
timeout -k 10 400 python3 bench.py "$@" > gpurun_out/b_$tag.json 2> gpurun_out/b_$tag.err \
  || { tail -30 gpurun_out/b_$tag.err; exit 1; }
cat gpurun_out/b_$tag.json; tail -5 gpurun_out/b_$tag.err
