#!/bin/bash
# Kernel-level profile of the C4 leg (bench.py --config c4, one timed step):
# rocprofv3 --kernel-trace --stats; prints the kernels of a few families.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/r05/prof_c4
rm -rf $o; mkdir -p $o
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $o -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 1 --warmup 0 > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
f=$(find $o -name "*kernel_stats.csv" | head -1)
grep -E "${FAM:-blur|noise|gray|black_resolve|rot_|border|center|move}" "$f" | cut -c1-220
