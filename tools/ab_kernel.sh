#!/bin/bash
# Per-kernel A/B of library builds: one-stream 128-page bench under
# rocprofv3 --kernel-trace --stats for each build in LIBS, then the average
# duration of the kernels matching KERN (regex); then ab_libs.sh's
# throughput A/B.  usage: LIBS="lib lib_x" KERN="noise" tools/ab_kernel.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abk
Q="--no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0"
for l in ${LIBS:-lib}; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/$l/libunpaper_hip.so timeout -s KILL 120 rocprofv3 --kernel-trace --stats \
    --output-format csv -d gpurun_out/abk/$l -- python3 bench.py $Q > gpurun_out/abk/$l.log 2>&1 || { tail -5 gpurun_out/abk/$l.log; exit 1; }
  python3 profiles/summarize.py gpurun_out/abk/$l 2 > gpurun_out/abk/$l.txt
  echo "== $l"; grep -E "${KERN:-.}" gpurun_out/abk/$l.txt | head -8
done
[ "${THROUGHPUT:-1}" = 1 ] && bash tools/ab_libs.sh
