#!/bin/bash
# Round-2 evidence on one GPU, each step under its own limit:
#  1. kernel trace + stats of the default bench command
#  2. FETCH_SIZE and WRITE_SIZE passes (separate) -> profiles/traffic.json
#  3. clock / VALU pass -> profiles/valu.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r02
mkdir -p $out
Q="--no-cpu --no-host-io --no-latency --no-verify --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -- \
  python3 bench.py --steps 5 --no-host-io --no-cpu > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
echo "trace done"; tail -1 $out/trace.log | cut -c1-200
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -- python3 bench.py $Q > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
echo "fetch done"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -- python3 bench.py $Q > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
echo "write done"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $out/clk -- python3 bench.py $Q > $out/clk.log 2>&1 || { tail -5 $out/clk.log; exit 1; }
echo "clock done"
python3 profiles/clock_table.py $out/clk 64 $out/valu.json > $out/clock_table.txt && head -25 $out/clock_table.txt
