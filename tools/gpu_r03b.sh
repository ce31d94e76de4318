#!/bin/bash
# runner / C-ABI GPU tests, then a 2-rank rehearsal of the driver's N>1 bench
# launch on the one GPU of the box (both ranks on device 0: LOCAL_RANK % ndev)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_runner_gpu.py tests/test_c_abi_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/gpu_runner.log 2>&1 || { tail -30 gpurun_out/gpu_runner.log; exit 1; }
tail -1 gpurun_out/gpu_runner.log
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu --no-host-io --no-c4 \
  > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail -20 gpurun_out/bench_n2.err; exit 1; }
tail -c 600 gpurun_out/bench_n2.json
