#!/bin/bash
# SQ counters per wave and HBM bytes of the C4 pipeline's kernels (4 sheets, one pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
Q="--config c4 --pages 4 --steps 1 --warmup 0 --no-verify --streams 1"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmcc4_sq -- python3 bench.py $Q > gpurun_out/pmcc4_sq.log 2>&1 || { tail -5 gpurun_out/pmcc4_sq.log; exit 1; }
python3 profiles/pmc_table.py "$(dirname $(find gpurun_out/pmcc4_sq -name '*counter_collection.csv' | head -1))" 10
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcc4_f -- python3 bench.py $Q > gpurun_out/pmcc4_f.log 2>&1 || { tail -5 gpurun_out/pmcc4_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcc4_w -- python3 bench.py $Q > gpurun_out/pmcc4_w.log 2>&1 || { tail -5 gpurun_out/pmcc4_w.log; exit 1; }
echo done
