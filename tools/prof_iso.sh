#!/bin/bash
# Isolated per-kernel times: one stream, 256 pages, batches of 32 sheets.
# usage (on the GPU box): tools/prof_iso.sh TAG   (env vars pass through)
set -e -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/iso_$tag -o run -- \
  python3 bench.py --no-cpu --pages 256 --steps 1 --warmup 1 --streams 1 --batch 32 \
  > gpurun_out/iso_$tag.json 2> gpurun_out/iso_$tag.err
python3 profiles/summarize.py gpurun_out/iso_$tag/run_results.db 16 > gpurun_out/iso_$tag.txt
