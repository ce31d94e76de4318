#!/bin/bash
# host-fed figure 2: DMA engines (default) vs shader copies (HSA_ENABLE_SDMA=0),
# the raw copy probe and the runner (bench host_io), 1 MI355X
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for sd in 1 0; do
  HSA_ENABLE_SDMA=$sd timeout -k 10 120 python3 tools/pcie_probe2.py > gpurun_out/probe2_sdma$sd.txt 2>&1 || { tail -3 gpurun_out/probe2_sdma$sd.txt; exit 1; }
  echo "SDMA=$sd"; cat gpurun_out/probe2_sdma$sd.txt
  for cfg in "32 8" "16 8" "8 16"; do
    set -- $cfg
    HSA_ENABLE_SDMA=$sd timeout -k 10 150 python3 bench.py --no-cpu --no-latency --no-c4 --probe 0 --steps 2 --warmup 1 --host-batch $1 --host-streams $2 > gpurun_out/hio_s${sd}_$1_$2.json 2>gpurun_out/hio.err || { tail -3 gpurun_out/hio.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/hio_s${sd}_$1_$2.json').read().strip().splitlines()[-1]); h=d['host_io']
print('SDMA=$sd batch $1 streams $2:', h['h2d_d2h']['value'], 'pages/s; pnm', h['pnm_write']['value'], '; resident', d['value'])"
  done
done
