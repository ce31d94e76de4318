#!/bin/bash
# Round-5 GPU checks on one box: `tools/gpu_r05.sh [pytest -k expr] [bench args]`
# runs the selected GPU tests, then (when BENCH=1) the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r05
mkdir -p $o
K="${1:-}"
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" \
    > $o/gpu_tests.log 2>&1 || { tail -40 $o/gpu_tests.log; exit 1; }
  tail -3 $o/gpu_tests.log
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
  tail -c 3000 $o/bench.json
fi
