#!/bin/bash
# A/B of an env switch under the default bench load: tools/ab_env.sh VAR [steps]
set -o pipefail
var=$1; steps=${2:-8}
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for mode in on off; do
    if [ $mode = off ]; then export $var=1; else unset $var; fi
    timeout -k 10 200 python3 bench.py --no-cpu --probe 0 --steps $steps > gpurun_out/ab_$mode$rep.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$mode$rep.json').read().strip().splitlines()[-1]); print('$var $mode', d['value'], d['ms_per_step'])"
  done
done
