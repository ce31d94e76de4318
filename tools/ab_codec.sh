#!/bin/bash
# Codec occupancy A/B (round 6): JP2 / JPEG runner legs and the host-fed
# jp2_write figure for the library builds named below (make lib VARIANT=...).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/t1
leg() { # lib config
  UNPAPER_HIP_LIB=unpaper-gpu_amd/$1/libunpaper_hip.so timeout -k 10 200 python3 bench.py --config $2 > gpurun_out/t1/$1_$2.json 2> gpurun_out/t1/$1_$2.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/t1/$1_$2.json').read().strip().splitlines()[-1]); print('$1 $2', d['value'], d.get('verified'))"
}
for l in lib lib_t1w5 lib_t1w7; do leg $l jp2; done
for l in lib lib_jd6 lib_jd8 lib; do leg $l jpeg; done
for l in lib lib_enc6; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/$l/libunpaper_hip.so timeout -k 10 300 python3 bench.py --no-c4 --no-cpu --no-latency --steps 3 > gpurun_out/t1/h_$l.json 2> gpurun_out/t1/h_$l.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/t1/h_$l.json').read().strip().splitlines()[-1]); h=d['host_io']; print('$l host', h['jp2_write']['value'], h['jpeg_write']['value'], d['value'])"
done
