set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in 0 256; do
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_DOUBLE=$v timeout -k 10 200 python3 bench.py --no-cpu --probe 0 --steps 5 > gpurun_out/cmp$v.json 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/cmp$v.json').read().strip().splitlines()[-1]); print('diag $v', d['value'], d['ms_per_step'])"
done
