set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for s in 4 8 12 16; do
  timeout -k 10 240 python3 bench.py --config c4 --no-latency --c4-streams $s > gpurun_out/c4s$s.json 2> gpurun_out/c4s$s.err || { tail -5 gpurun_out/c4s$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4s$s.json').read().strip().splitlines()[-1]); print('streams $s', d['value'], d.get('verified'), d.get('mismatches'), d.get('ms_per_step'))"
done
