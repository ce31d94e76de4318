set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filters_gpu.py tests/test_pipeline_gpu.py > gpurun_out/black_tests.log 2>&1 || { tail -30 gpurun_out/black_tests.log; exit 1; }
tail -2 gpurun_out/black_tests.log
for v in old new; do
  cp ab/$v.so unpaper-gpu_amd/lib/libunpaper_hip.so
  timeout -k 10 200 python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --probe 0 --steps 2 --warmup 1 --streams 1 --pages 128 --stages > gpurun_out/stages_$v.json 2> gpurun_out/stages_$v.txt || exit 1
  echo "== $v"; grep -E "black|noise|rotate" gpurun_out/stages_$v.txt
done
cp ab/new.so unpaper-gpu_amd/lib/libunpaper_hip.so
bash tools/ab_lib.sh 2
UNPAPER_HIP_LIB=unpaper-gpu_amd/lib_diag/libunpaper_hip.so UPHIP_DIAG_NOISE=16 timeout -k 10 200 python3 bench.py --tuning --no-cpu --no-host-io --no-latency --no-verify --probe 0 --pages 8 --batch 8 --streams 1 --steps 1 --warmup 0 > gpurun_out/bk.log 2>&1 || exit 1
grep "uphip black" gpurun_out/bk.log | head -4
