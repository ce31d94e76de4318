#!/bin/bash
# Round-6 probe: selected GPU tests, the blackfilter replay counters of the
# tuning build (one C3 batch, C4 sheets 1 and 13), then the JPEG / JPEG 2000
# runner legs under rocprofv3 (kernel table).  Writes gpurun_out/r06p/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r06p
mkdir -p $o
if [ -n "${K:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" \
    > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
  tail -2 $o/gpu_tests.log
fi
if [ "${BLACK:-0}" = 1 ]; then
  Q="--tuning --no-cpu --no-host-io --no-latency --no-verify --pages 64 --steps 1 --warmup 0 --streams 1 --probe 0"
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 300 \
    python3 bench.py $Q > $o/black_diag.txt 2>&1 || { tail -5 $o/black_diag.txt; exit 1; }
  grep "uphip black" $o/black_diag.txt | sort | uniq -c | sort -rn | head -12
fi
for c in ${CFG:-}; do
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_$c -- python3 $R/bench.py --config $c ${PAGES:+--pages $PAGES} > $o/bench_$c.json 2> $o/bench_$c.err || { tail -20 $o/bench_$c.err; exit 1; }
  tail -c 700 $o/bench_$c.json
  f=$(find $o/prof_$c -name "*kernel_stats.csv" | head -1)
  grep -i "noise\|black_resolve\|t1\|Name" "$f" | cut -c1-60,150-400 | head -8
  cd $R
done
