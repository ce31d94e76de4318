#!/bin/bash
# GPU tests only: a -k selection (or all), logged under gpurun_out/.
# usage: tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
tag=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
sel=()
[ -n "$2" ] && sel=(-k "$2")
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${sel[@]}" \
  > gpurun_out/t_$tag.log 2>&1 || { grep -E "PASS|FAIL|Error" gpurun_out/t_$tag.log | tail -30; tail -40 gpurun_out/t_$tag.log; exit 1; }
tail -3 gpurun_out/t_$tag.log
