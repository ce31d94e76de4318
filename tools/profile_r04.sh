#!/bin/bash
# Round-4 evidence on one GPU, each step under its own limit (writes gpurun_out/r04/;
# the summaries copied into profiles/r04/ name this script in their header):
#  1. kernel trace + stats of the default bench command (16 streams)
#  2. one-stream kernel trace (128 pages) -> per-kernel table per 64-sheet launch
#  3. FETCH_SIZE and WRITE_SIZE passes (separate) -> traffic.json (pipeline + rotate)
#  4. clock / VALU pass -> valu.json
#  5. the C4 bilinear rotate's FETCH/WRITE passes (tools/traffic_c4.sh) -> tc4/c4.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r04
mkdir -p $out
Q="--no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -- \
  python3 bench.py --steps 5 --no-host-io --no-cpu --no-c4 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
echo "trace done"; tail -1 $out/trace.log | cut -c1-200
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/iso -- python3 bench.py $Q > $out/iso.log 2>&1 || { tail -5 $out/iso.log; exit 1; }
python3 profiles/summarize.py $out/iso 2 > $out/kernel_stats_1stream.txt && head -45 $out/kernel_stats_1stream.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -- python3 bench.py $Q > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
echo "fetch done"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -- python3 bench.py $Q > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
echo "write done"
cp profiles/traffic.json $out/traffic.json
python3 profiles/traffic.py $out/fetch $out/write k_rotate_cubic_g8f deskew_rotate 1113579520 64 128 $out/traffic.json | tail -8
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $out/clk -- python3 bench.py $Q > $out/clk.log 2>&1 || { tail -5 $out/clk.log; exit 1; }
echo "clock done"
python3 profiles/clock_table.py $out/clk 64 $out/valu.json > $out/clock_table.txt && head -30 $out/clock_table.txt
tools/traffic_c4.sh > $out/tc4.log 2>&1 || { tail -5 $out/tc4.log; exit 1; }
python3 profiles/traffic.py --merge-c4 gpurun_out/tc4/c4.json $out/traffic.json
