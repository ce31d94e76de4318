#!/bin/bash
# full GPU suite, then a 1-stream C3 kernel trace summary, then the default
# bench line (C3 + C4 values and verification)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/chk; rm -rf $out; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tr -- python3 bench.py --no-cpu --no-host-io --no-latency --no-verify --no-c4 --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0 > $out/tr.log 2>&1 || { tail -5 $out/tr.log; exit 1; }
python3 profiles/summarize.py $out/tr 2 | head -24
timeout -k 10 300 python3 bench.py --no-cpu --no-host-io --no-latency > $out/b.json 2> $out/b.err || { tail $out/b.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/b.json').read().strip().splitlines()[-1]); c=d['c4']
print('C3', d['value'], d['verified'], d['mismatches'], 'C4', c['value'], c['verified'], c['mismatches'])"
