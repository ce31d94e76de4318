#!/bin/bash
# A/B of library builds on the JPEG 2000 paths: tools/j2k_bench.py (one page
# decode / encode) and bench.py --config jp2 (runner) per build in LIBS.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/j2k
for l in ${LIBS:-lib}; do
  echo "== $l"
  UNPAPER_HIP_LIB=unpaper-gpu_amd/$l/libunpaper_hip.so timeout -k 10 300 python3 tools/j2k_bench.py ${PAGES:-2} \
    > gpurun_out/j2k/ab_$l.txt 2>&1 || { tail -5 gpurun_out/j2k/ab_$l.txt; exit 1; }
  cat gpurun_out/j2k/ab_$l.txt
  UNPAPER_HIP_LIB=unpaper-gpu_amd/$l/libunpaper_hip.so timeout -k 10 300 python3 bench.py --config jp2 \
    --pages ${RPAGES:-256} > gpurun_out/j2k/ab_$l.json 2> gpurun_out/j2k/ab_$l.err || { tail -5 gpurun_out/j2k/ab_$l.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/j2k/ab_$l.json').read().strip().splitlines()[-1]); print('$l runner', d['value'], 'pages/s verified', d['verified'])"
done
