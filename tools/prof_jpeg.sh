#!/bin/bash
# Kernel-level profile of the JPEG runner legs: bench.py --config jpeg
# (device Huffman decode) under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/r05/prof_jpeg
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -- python3 $GRAFT_REPO_ROOT/bench.py --config jpeg --pages ${PAGES:-64} > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 1; }
tail -c 600 $o/bench.json
f=$(find $o -name "*kernel_stats.csv" | head -1)
echo "$f"
head -25 "$f"
