#!/bin/bash
# rocprofv3 PMC passes over the pipeline (one stream, 128 A4 pages = two
# 64-sheet batches, product library), one pass per counter group, each under
# its own time limit.  Writes gpurun_out/pmc_TAG_N/ and prints per-kernel tables.
# usage: tools/pmc_passes.sh TAG "COUNTERS PASS 1" ["COUNTERS PASS 2" ...]
set -o pipefail
tag=${1:-x}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
n=0
for C in "$@"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${tag}_$n -- \
    python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --pages 128 --steps 1 --warmup 0 \
    --streams 1 --probe 0 > gpurun_out/pmc_${tag}_$n.log 2>&1 || { tail -5 gpurun_out/pmc_${tag}_$n.log; exit 1; }
  python3 profiles/pmc_summary.py "$(dirname $(find gpurun_out/pmc_${tag}_$n -name '*counter_collection.csv' | head -1))" > gpurun_out/pmc_${tag}_$n.txt
  echo "pass $n: $C"; head -60 gpurun_out/pmc_${tag}_$n.txt
done
