#!/bin/bash
# Instruction counts of k_rotate_cubic_g8f per wave for timing-only variants of
# the tuning build (tools/rot_variants.sh bits): where the VALU/SALU/LDS
# instructions of the rotate go.  usage: VARIANTS="0 512 1536" tools/pmc_rot_variants.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-0 512 1536}; do
  UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_DOUBLE=$v timeout -s KILL 120 \
    rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
    --kernel-include-regex rotate_cubic --output-format csv -d gpurun_out/prv_$v -- \
    python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --pages 128 --steps 1 --warmup 0 \
    --no-c4 --streams 1 --probe 0 > gpurun_out/prv_$v.log 2>&1 || { tail -5 gpurun_out/prv_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
f = glob.glob(f"gpurun_out/prv_{v}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if "rotate_cubic_g8fILb0" in r["Kernel_Name"] or "k_rotate_cubic_g8f<false>" in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
w = acc["SQ_WAVES"] or 1
print("variant %s: waves %d  per wave: VALU %.0f SALU %.0f LDS %.0f SMEM %.0f" % (
    v, w, acc["SQ_INSTS_VALU"] / w, acc["SQ_INSTS_SALU"] / w, acc["SQ_INSTS_LDS"] / w, acc["SQ_INSTS_SMEM"] / w))
PY
done
