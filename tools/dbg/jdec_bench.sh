#!/bin/bash
# Builds tools/dbg/jdec_bench (here) or, with "run", makes 16 synthetic A4
# q95 pages and times the device Huffman decode on the GPU box.
set -e -o pipefail
cd "$(dirname "$0")/../.."
if [ "$1" != run ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iunpaper-gpu_amd/csrc -Iinclude \
    tools/dbg/jdec_bench.cpp -o tools/dbg/_jdec_bench -Lunpaper-gpu_amd/lib -lunpaper_hip \
    -Wl,-rpath,'$ORIGIN/../../unpaper-gpu_amd/lib'
  exit 0
fi
d=$(mktemp -d /dev/shm/jdb.XXXX)
python3 - "$d" <<'PY'
import sys, ctypes, numpy as np
from PIL import Image
L = ctypes.CDLL("unpaper-gpu_amd/lib/libunpaper_hip.so")
W, H = 2480, 3508
for i in range(16):
    g = np.empty((H, W), np.uint8)
    L.uphip_synth_page_host(ctypes.c_void_p(g.ctypes.data), W, W, H, i)
    Image.fromarray(g).save("%s/p%02d.jpg" % (sys.argv[1], i), "JPEG", quality=95)
PY
o=gpurun_out/jdb
mkdir -p $o
shift
timeout -k 10 120 tools/dbg/_jdec_bench ${1:-16} ${2:-5} $d/*.jpg | tee $o/run.json
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$o/prof \
    -- $GRAFT_REPO_ROOT/tools/dbg/_jdec_bench ${1:-16} ${2:-5} $d/*.jpg > /dev/null
  cat $(find $GRAFT_REPO_ROOT/$o/prof -name '*kernel_stats.csv') | cut -c1-150
fi
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  n=0
  for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_LDS" \
           "SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT SQ_INSTS_VMEM_WR"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/$o/pmc$n \
      -- $GRAFT_REPO_ROOT/tools/dbg/_jdec_bench ${1:-16} 1 $d/*.jpg > /dev/null
    python3 $GRAFT_REPO_ROOT/profiles/pmc_summary.py "$(dirname $(find $GRAFT_REPO_ROOT/$o/pmc$n -name '*counter_collection.csv' | head -1))" | tee $GRAFT_REPO_ROOT/$o/pmc$n.txt
  done
fi
rm -rf "$d"
