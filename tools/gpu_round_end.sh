#!/bin/bash
# One-call round evidence with an A/B gate: parity of ab/new.so on the
# pipeline/op tests, a 2x load A/B against ab/old.so, keep the faster build,
# then the full GPU suite, the default bench, the C4 mode and the rocprof
# passes of tools/profile_r02.sh on the kept build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/ab_check.sh 2 > gpurun_out/re_ab.txt 2>&1 || { tail -30 gpurun_out/re_ab.txt; exit 1; }
cat gpurun_out/re_ab.txt
keep=$(python3 - <<'PY'
import re
v = {"old": [], "new": []}
for line in open("gpurun_out/re_ab.txt"):
    m = re.match(r"^(old|new) ([0-9.]+)$", line.strip())
    if m: v[m.group(1)].append(float(m.group(2)))
o, n = sum(v["old"]) / len(v["old"]), sum(v["new"]) / len(v["new"])
print("new" if n > o * 1.002 else "old")
PY
) || exit 1
echo "kept build: $keep"
cp ab/$keep.so unpaper-gpu_amd/lib/libunpaper_hip.so
echo "$keep" > gpurun_out/re_kept.txt
bash tools/gpu_final.sh re || exit 1
bash tools/profile_r02.sh || exit 1
