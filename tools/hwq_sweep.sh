set -o pipefail
cd "$GRAFT_REPO_ROOT"
for cfg in "24 16" "24 20" "32 24" "32 32" "24 16"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --no-cpu --probe 0 --steps 6 --hw-queues $1 --streams $2 > gpurun_out/hwq.json 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/hwq.json').read().strip().splitlines()[-1]); print('hwq $1 streams $2', d['value'])"
done
