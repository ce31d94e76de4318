#!/bin/bash
# parity tests for the black filter, then replay counters on C3 band pages and C4 sheets
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filters_gpu.py tests/test_pipeline_gpu.py > gpurun_out/bb_tests.log 2>&1 || { tail -30 gpurun_out/bb_tests.log; exit 1; }
tail -1 gpurun_out/bb_tests.log
bash tools/black_exp.sh 16 | grep "uphip black:"
bash tools/black_c4.sh
timeout -k 10 200 python3 bench.py --config c4 --steps 3 > gpurun_out/c4_bb.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/c4_bb.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['latency_ms'], d['stages_ms_per_step']['blackfilter'])"
