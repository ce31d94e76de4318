#!/bin/bash
# Full GPU test suite, then the C4 bench mode and a host-I/O sweep.
set -o pipefail
tag=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/full_$tag.log 2>&1 || { tail -40 gpurun_out/full_$tag.log; exit 1; }
tail -3 gpurun_out/full_$tag.log
timeout -k 10 300 python3 bench.py --config c4 --steps 3 > gpurun_out/c4_$tag.json 2> gpurun_out/c4_$tag.err \
  || { tail -30 gpurun_out/c4_$tag.err; exit 1; }
cat gpurun_out/c4_$tag.json
for cfg in "32 4" "32 8" "64 4" "16 8"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu --no-latency --probe 0 --no-verify \
    --host-batch $1 --host-streams $2 > gpurun_out/hio_$tag_$1_$2.json 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/hio_$tag_$1_$2.json').read().strip().splitlines()[-1]); print('host', '$1x$2', d['host_io']['h2d_d2h'], d['host_io']['pnm_write']['value'])"
done
