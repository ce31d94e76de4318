#!/bin/bash
# SQ counters of the rotation kernels (new float-window vs old byte-window).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
for v in 0 512 1536; do
  UPHIP_DIAG_DOUBLE=$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_rot$v -- \
    python3 bench.py --no-cpu --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0 > gpurun_out/pmc_rot$v.log 2>&1 || exit 1
  python3 profiles/pmc_table.py "$(dirname $(find gpurun_out/pmc_rot$v -name '*counter_collection.csv' | head -1))" 3
done
