#!/bin/bash
# SQ counters per wave of the pipeline's top kernels (one stream, 128 pages).
# usage: tools/pmc_rot.sh TAG [UPHIP_DIAG_DOUBLE value]
set -o pipefail
tag=${1:-x}; v=${2:-0}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_DOUBLE=$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$tag -- \
  python3 bench.py --no-cpu --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0 > gpurun_out/pmc_$tag.log 2>&1 || exit 1
python3 profiles/pmc_table.py "$(dirname $(find gpurun_out/pmc_$tag -name '*counter_collection.csv' | head -1))" 12
