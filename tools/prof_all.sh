#!/bin/bash
# Round profile set (on the GPU box): kernel-trace stats of the default bench
# command, isolated per-kernel times (one stream), and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) behind roofline.traffic.   usage: tools/prof_all.sh TAG
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/pa_$tag
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/bench -o run -- python3 bench.py --no-cpu \
  > $o/bench.json 2> $o/bench.err || { tail $o/bench.err; exit 1; }
python3 profiles/summarize.py $o/bench 64 --last k_rotate_cubic_g8f 3 > $o/bench.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $o/iso -o run -- \
  python3 bench.py --no-cpu --pages 256 --steps 1 --warmup 1 --streams 1 --batch 64 --probe 0 \
  > $o/iso.json 2> $o/iso.err || { tail $o/iso.err; exit 1; }
python3 profiles/summarize.py $o/iso 8 > $o/iso.txt 2>&1 || true
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $o/pmc_$c -o run --output-format csv -- \
    python3 bench.py --pages 128 --steps 1 --warmup 1 --streams 1 --batch 64 --no-cpu --probe 0 \
    > $o/pmc_$c.log 2>&1 || { tail $o/pmc_$c.log; exit 1; }
done
cat $o/bench.json; head -40 $o/bench.txt; head -30 $o/iso.txt
