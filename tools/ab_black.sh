#!/bin/bash
# A/B of blackfilter replay builds: per-sheet replay counters (tuning builds
# DLIBS) and the one-stream kernel table (product-like builds LIBS) on one C3
# batch.  usage: DLIBS="lib_diag lib_diagold" LIBS="lib lib_old" tools/ab_black.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
o=$R/gpurun_out/r06ab
mkdir -p $o
Q="--no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0"
for l in ${DLIBS:-}; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/$l/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 \
    python3 bench.py $Q --tuning > $o/diag_$l.txt 2>&1 || { tail -5 $o/diag_$l.txt; exit 1; }
  echo "== $l"; grep "uphip black" $o/diag_$l.txt | head -3
done
cd /tmp && export TMPDIR=/tmp
for l in ${LIBS:-}; do
  UNPAPER_HIP_LIB=$R/unpaper-gpu_amd/$l/libunpaper_hip.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/iso_$l -- python3 $R/bench.py $Q --tuning > $o/iso_$l.log 2>&1 || { tail -5 $o/iso_$l.log; exit 1; }
  echo "== $l"; python3 $R/profiles/summarize.py $o/iso_$l 2 | grep -E "black_resolve|pipeline kernels"
done
