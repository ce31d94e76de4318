#!/bin/bash
# Round-4 closing evidence on one GPU: smoke, the GPU suite, the default bench
# line exactly as the driver runs it (CPU baseline included), and the driver's
# N>1 launch rehearsed with two ranks on this one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/final
o=gpurun_out/final
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 \
  || { tail -30 $o/smoke.log; exit 1; }
cat $o/smoke.log
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $o/gpu_tests.log 2>&1 || { tail -30 $o/gpu_tests.log; exit 1; }
tail -2 $o/gpu_tests.log
timeout -k 10 400 python3 bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$o/bench.json').read().strip().splitlines()[-1]); c=d['c4']
print('C3', d['value'], d['verified'], d['mismatches'], 'frac', d['roofline']['frac'], 'pipe', d['roofline']['pipeline_frac'], 'cpu', d['cpu_baseline']['value'] if d['cpu_baseline'] else None, 'C4', c['value'], c['verified'], c['mismatches'], 'hio', d['host_io']['h2d_d2h']['value'])"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > $o/bench_n2.json 2> $o/bench_n2.err \
  || { tail -20 $o/bench_n2.err; exit 1; }
python3 -c "
import json; L=[l for l in open('$o/bench_n2.json') if l.startswith('{')]; d=json.loads(L[-1]); print('N2', d['value'], d['verified'], d['mismatches'], d['valid'])"
