cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 4 --batch 4 --streams 1 --steps 1 --warmup 0 > gpurun_out/bk2.log 2>&1 || { tail gpurun_out/bk2.log; exit 1; }
grep -c "^miss" gpurun_out/bk2.log
