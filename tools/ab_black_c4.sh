#!/bin/bash
# Blackfilter replay counters of tuning builds on C4 (all 16 sheets, one pass)
# and one C3 batch.  usage: DLIBS="lib_diag lib_diagr05" tools/ab_black_c4.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/r06c4
mkdir -p $o
for l in ${DLIBS:-lib_diag}; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/$l/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 \
    python3 bench.py --config c4 --tuning --steps 1 --warmup 0 --no-verify --no-latency > $o/c4_$l.txt 2>&1 || { tail -5 $o/c4_$l.txt; exit 1; }
  echo "== $l"; grep "uphip black" $o/c4_$l.txt | sort -t' ' -k6 -n -r | head -4
done
