#!/usr/bin/env python3
"""Build profiles/traffic.json (HBM bytes per launch / per page) from two
rocprofv3 --pmc passes of the same command: one with FETCH_SIZE, one with
WRITE_SIZE (they do not fit in one pass on gfx950).

usage: traffic.py <fetch-pass dir> <write-pass dir> <kernel-substring> <stage> \
                  <alg-bytes-per-launch> <pages-per-launch> <pages-in-run> [out.json]

Besides the named kernel it sums every pipeline dispatch of the run (all
kernels except the synthetic-page generator) into HBM bytes per page: the
whole-pipeline FETCH+WRITE figure bench.py reports as
roofline.pipeline_hbm_bytes_per_page.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
in KiB; FETCH_SIZE tallies half of the bytes of coalesced streaming reads on
gfx950, so it is doubled; WRITE_SIZE is exact.  The doubling was re-checked
on this pipeline's k_copy (16 B/lane) and k_colsum_g (4 B/lane) reads; the
same pass also carries those kernels, so the check is printed each time.
"""
import collections
import csv
import glob
import json
import os
import sys


def dispatches(path, counter):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def per_launch(path, counter):
    return {k: sum(v) / len(v) for k, v in dispatches(path, counter).items()}


def pipeline_total(path, counter):
    return sum(sum(v) for k, v in dispatches(path, counter).items() if "synth" not in k)


def pick(d, sub):
    ks = [k for k in d if sub in k]
    if not ks:
        raise SystemExit("no kernel matching %r" % sub)
    return max(d[k] for k in ks)  # the full-plane variant


def merge_c4(path, out):
    with open(path) as f:
        c4 = json.load(f)
    try:
        with open(out) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        doc = {}
    if os.environ.get("TRAFFIC_COMMIT"):
        c4["library_commit"] = os.environ["TRAFFIC_COMMIT"]
    doc["c4"] = c4
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print("c4 merged into", out)


def main():
    if sys.argv[1] == "--merge-c4":
        merge_c4(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else
                 os.path.join(os.path.dirname(__file__), "traffic.json"))
        return
    fdir, wdir, kern, stage, alg, pages, run_pages = sys.argv[1:8]
    out = sys.argv[8] if len(sys.argv) > 8 else os.path.join(os.path.dirname(__file__), "traffic.json")
    alg, pages, run_pages = int(alg), int(pages), int(run_pages)
    fetch, write = per_launch(fdir, "FETCH_SIZE"), per_launch(wdir, "WRITE_SIZE")
    for ref in ("k_copy", "k_colsum_g"):
        try:
            print("calibration %-10s FETCH raw %.1f MB/launch, doubled %.1f MB" %
                  (ref, pick(fetch, ref) / 1e6, 2 * pick(fetch, ref) / 1e6))
        except SystemExit:
            pass
    fr, wr = pick(fetch, kern), pick(write, kern)
    hbm = 2 * fr + wr
    name = kern.split("(")[0].split("::")[-1]
    doc = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-trace "
                  "-- python3 bench.py --pages 128 --steps 1 --warmup 0 --streams 1 --probe 0 "
                  "--no-cpu --no-host-io --no-latency --no-verify (tools/pmc_passes.sh); "
                  "1 MI355X; %d sheets per launch" % pages,
        "correction": "FETCH_SIZE x2 (gfx950 tallies half of coalesced streaming reads); "
                      "counter values are KiB",
        "kernels": {name: {"fetch_raw_bytes_per_launch": int(fr),
                           "write_bytes_per_launch": int(wr),
                           "hbm_bytes_per_launch": int(hbm),
                           "alg_bytes_per_launch": alg}},
        "bytes_per_page": {stage: int(hbm / pages)},
    }
    pf, pw = pipeline_total(fdir, "FETCH_SIZE"), pipeline_total(wdir, "WRITE_SIZE")
    doc["pipeline_fetch_bytes_per_page"] = int(2 * pf / run_pages)
    doc["pipeline_write_bytes_per_page"] = int(pw / run_pages)
    doc["pipeline_bytes_per_page"] = int((2 * pf + pw) / run_pages)
    doc["pipeline_pages_in_run"] = run_pages
    print("pipeline: fetch x2 %.1f MB + write %.1f MB = %.1f MB per page" %
          (2 * pf / run_pages / 1e6, pw / run_pages / 1e6, (2 * pf + pw) / run_pages / 1e6))
    # keys other tools own (the C4 rotate's "c4", tools/traffic_c4.sh) survive
    try:
        with open(out) as f:
            old = json.load(f)
        for k, v in old.items():
            doc.setdefault(k, v)
    except (OSError, ValueError):
        pass
    # the library the passes measured (the GPU box gets no .git: the caller
    # passes the commit) and the script that ran them
    for key, env in (("library_commit", "TRAFFIC_COMMIT"), ("script", "TRAFFIC_SCRIPT")):
        if os.environ.get(env):
            doc[key] = os.environ[env]
    if os.environ.get("TRAFFIC_SCRIPT"):
        doc["source"] = doc["source"].replace("tools/pmc_passes.sh", os.environ["TRAFFIC_SCRIPT"])
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print("%s: fetch %.1f MB (x2 %.1f) + write %.1f MB = %.1f MB/launch vs alg %.1f MB (%.3fx)" %
          (name, fr / 1e6, 2 * fr / 1e6, wr / 1e6, hbm / 1e6, alg / 1e6, hbm / alg))


if __name__ == "__main__":
    main()
