#!/bin/bash
# C4 parity over all 16 hashed sheets, the filter suites, and the VALU table
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_runner_gpu.py tests/test_filters_gpu.py > gpurun_out/c4p.log 2>&1 || { tail -30 gpurun_out/c4p.log; exit 1; }
tail -1 gpurun_out/c4p.log
timeout -k 10 200 python3 bench.py --config c4 --steps 3 > gpurun_out/c4_v.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/c4_v.json').read().strip().splitlines()[-1]); print('c4', d['value'], 'verified', d['verified'], 'mismatches', d['mismatches'])"
bash tools/pmc_clock.sh v | grep -E "blur_counts|gray_cells|rowsum|colsum"
