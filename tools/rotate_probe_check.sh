#!/bin/bash
# The bench line's roofline launch time against rocprofv3: the default C3
# bench (CPU, host-I/O, C4 and latency legs off) under --kernel-trace
# --stats; the last three k_rotate_cubic_g8f<false> dispatches are the
# line's three isolated probe launches, whose average must agree with its
# roofline.avg_launch_ms.  Writes gpurun_out/rpc/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
o=gpurun_out/rpc
mkdir -p $o
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -- python3 bench.py --no-cpu --no-host-io --no-c4 --no-latency > $o/bench.json 2> $o/bench.err || { tail -5 $o/bench.err; exit 1; }
python3 - <<'PY'
import csv, glob, json
o = "gpurun_out/rpc"
line = json.loads(open(o + "/bench.json").read().strip().splitlines()[-1])
tr = glob.glob(o + "/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(tr)) if "k_rotate_cubic_g8f<false>" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[-3:]]
st = glob.glob(o + "/prof/**/*kernel_stats.csv", recursive=True)[0]
avg_all = [r for r in csv.DictReader(open(st)) if "k_rotate_cubic_g8f<false>" in r["Name"]][0]
out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --no-host-io --no-c4 --no-latency",
       "bench_value": line["value"], "bench_avg_launch_ms": line["roofline"]["avg_launch_ms"],
       "rocprof_last3_ms": [round(x, 4) for x in last], "rocprof_last3_avg_ms": round(sum(last) / 3, 4),
       "rocprof_all_launches": int(avg_all["Calls"]), "rocprof_all_avg_ms": round(float(avg_all["AverageNs"]) / 1e6, 4),
       "note": "the timed region runs 16 batches at once (all-launch average includes concurrent launches); the line's roofline uses the 3 isolated probes"}
json.dump(out, open(o + "/rotate_probe_check.json", "w"), indent=1)
print(json.dumps(out))
PY
