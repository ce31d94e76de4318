#!/bin/bash
# Copy the summaries of a tools/prof_all.sh run (gpurun_out/pa_TAG, merged
# back from the GPU box) into profiles/.   usage: tools/collect_profiles.sh TAG
set -e -o pipefail
tag=${1:?tag}
P=profiles
O=gpurun_out/pa_$tag
val() { python3 -c "import json; d=json.load(open('$O/bench.json')); print($1)"; }
{
  echo "# rocprofv3 --kernel-trace --stats -d $O/bench -o run -- python3 bench.py --no-cpu   (tools/prof_all.sh $tag)"
  echo "# 1 MI355X; 1000 pages, 1 warm-up + 3 timed steps of 16 batch launches of 64 sheets + 3 probe launches;"
  echo "# streams $(val "d['config']['streams']"), HW queues $(val "d['config']['hw_queues']"); durations overlap across streams"
  echo "# bench value under the profiler: $(val "d['value']") pages/s; bench roofline.avg_launch_ms $(val "d['roofline']['avg_launch_ms']")"
  cat $O/bench.txt
} > $P/r01_kernel_summary.txt
{
  echo "# rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --pages 256 --steps 1 --warmup 1 --streams 1 --batch 64 --probe 0   (tools/prof_all.sh $tag)"
  echo "# one stream, 8 launches of 64 sheets: isolated per-kernel times"
  cat $O/iso.txt
} > $P/r01_kernel_isolated_1stream.txt
cp $O/bench.json $P/r01_bench_under_rocprof.json
python3 profiles/traffic.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE k_rotate_cubic_g8f deskew_rotate \
  $((2 * 2480 * 3508 * 64)) 64 $P/traffic.json | tail -1
sed -i 's/32 sheets per launch/64 sheets per launch/; s/--streams 1 --no-cpu;/--streams 1 --batch 64 --no-cpu --probe 0;/' \
  $P/traffic.json
head -4 $P/r01_kernel_summary.txt
tail -1 $P/r01_kernel_summary.txt
