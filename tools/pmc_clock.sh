#!/bin/bash
# Effective shader clock and VALU counts per kernel: GRBM_GUI_ACTIVE and SQ
# counters with the kernel trace (durations), one stream, 128 A4 pages.
set -o pipefail
tag=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/clk_$tag -- \
  python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --pages 128 --steps 1 --warmup 0 --no-c4 \
  --streams 1 --probe 0 > gpurun_out/clk_$tag.log 2>&1 || { tail -5 gpurun_out/clk_$tag.log; exit 1; }
python3 profiles/clock_table.py gpurun_out/clk_$tag > gpurun_out/clk_$tag.txt && rm -rf gpurun_out/clk_$tag && head -16 gpurun_out/clk_$tag.txt
