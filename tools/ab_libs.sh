#!/bin/bash
# A/B of library builds (make lib VARIANT=name ...; "lib" = the product build):
# the default C3 bench without the C4 / CPU / host-I/O / latency legs, each
# build twice in alternation; prints pages/s and the isolated rotate launch.
# usage: LIBS="lib lib_m6" tools/ab_libs.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for l in ${LIBS:-lib}; do
    UNPAPER_HIP_LIB=unpaper-gpu_amd/$l/libunpaper_hip.so timeout -k 10 200 \
      python3 bench.py --no-cpu --no-c4 --no-host-io --no-latency --probe 5 --steps 10 \
      > gpurun_out/ab_$l.json 2> gpurun_out/ab_$l.err || { tail -5 gpurun_out/ab_$l.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$l.json').read().strip().splitlines()[-1]); print('$l', d['value'], 'pages/s rotate', d['roofline']['avg_launch_ms'], 'ms verified', d['verified'], d['mismatches'])"
  done
done
