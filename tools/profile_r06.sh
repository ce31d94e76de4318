#!/bin/bash
# Round-6 evidence on the final library (writes gpurun_out/r06e/):
#  1. one-stream kernel trace of 128 C3 pages -> per-kernel table a 64-sheet launch
#  2. clock / VALU / SALU pass -> clock_table.txt, valu.json (clocks only from
#     dispatches >= 0.3 ms, profiles/clock_table.py)
#  3. FETCH_SIZE and WRITE_SIZE passes (separate) -> traffic.json (rotate and
#     whole-pipeline bytes per page), stamped with COMMIT
#  4. the C4 bilinear rotate's FETCH / WRITE passes merged into it
# usage (from the build container): gpurun -- "COMMIT=$(git rev-parse --short HEAD) tools/profile_r06.sh"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06e
mkdir -p $out
export TRAFFIC_COMMIT="${COMMIT:-unknown}" TRAFFIC_SCRIPT="tools/profile_r06.sh"
Q="--no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/iso -- python3 bench.py $Q > $out/iso.log 2>&1 || { tail -5 $out/iso.log; exit 1; }
python3 profiles/summarize.py $out/iso 2 > $out/kernel_stats_1stream.txt && head -30 $out/kernel_stats_1stream.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $out/clk -- python3 bench.py $Q > $out/clk.log 2>&1 || { tail -5 $out/clk.log; exit 1; }
python3 profiles/clock_table.py $out/clk 64 $out/valu.json > $out/clock_table.txt && head -16 $out/clock_table.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/fetch -- python3 bench.py $Q > $out/fetch.log 2>&1 || { tail -5 $out/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/write -- python3 bench.py $Q > $out/write.log 2>&1 || { tail -5 $out/write.log; exit 1; }
cp profiles/traffic.json $out/traffic.json
python3 profiles/traffic.py $out/fetch $out/write k_rotate_cubic_g8f deskew_rotate 1113579520 64 128 $out/traffic.json | tail -6
tools/traffic_c4.sh | tail -3 && python3 profiles/traffic.py --merge-c4 gpurun_out/tc4/c4.json $out/traffic.json
