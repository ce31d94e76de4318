#!/bin/bash
# Round-6 GPU checks on one box (writes gpurun_out/r06/):
#   K="expr"      run the GPU tests selected by -k expr ("all": the whole suite)
#   BENCH=1       the default bench line (BENCH_ARGS adds flags)
#   CFG="jpeg jp2 pdf"  bench --config <c> legs, each under rocprofv3 --kernel-trace --stats
#                 (PAGES= pages each)
#   ISO=1         one-stream kernel trace of 128 C3 pages (per-kernel table a 64-sheet launch)
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r06${TAG:+_$TAG}
mkdir -p $o
if [ -n "${K:-}" ]; then
  if [ "$K" = all ]; then sel=(); else sel=(-k "$K"); fi
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "${sel[@]}" \
    > $o/gpu_tests.log 2>&1 || { tail -40 $o/gpu_tests.log; exit 1; }
  tail -3 $o/gpu_tests.log
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
  tail -c 4000 $o/bench.json
fi
if [ "${ISO:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  Q="--no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/iso -- python3 $R/bench.py $Q > $o/iso.log 2>&1 || { tail -5 $o/iso.log; exit 1; }
  python3 $R/profiles/summarize.py $o/iso 2 > $o/kernel_stats_1stream.txt && head -45 $o/kernel_stats_1stream.txt
  cd $R
fi
for c in ${CFG:-}; do
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$c -- python3 $R/bench.py --config $c ${PAGES:+--pages $PAGES} > $o/bench_$c.json 2> $o/bench_$c.err || { tail -20 $o/bench_$c.err; exit 1; }
  tail -c 1500 $o/bench_$c.json
  f=$(find $o/prof_$c -name "*kernel_stats.csv" | head -1)
  head -16 "$f"
  cd $R
done
