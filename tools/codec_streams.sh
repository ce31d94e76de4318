#!/bin/bash
# JPEG / JPEG 2000 runner lines over (sheets per batch, batches in flight)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cs
for cfg in ${CFGS:-"jp2 32 8" "jp2 32 16" "jp2 64 8" "jp2 16 16" "jpeg 32 8" "jpeg 32 16"}; do
  set -- $cfg
  timeout -k 10 240 python3 bench.py --config $1 --pages 512 --host-batch $2 --codec-streams $3 \
    > gpurun_out/cs/$1_$2_$3.json 2> gpurun_out/cs/$1_$2_$3.err || { tail -5 gpurun_out/cs/$1_$2_$3.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cs/$1_$2_$3.json').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['verified'])"
done
