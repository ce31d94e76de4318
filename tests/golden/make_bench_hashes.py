#!/usr/bin/env python3
"""Generate tests/golden/bench_hashes.json: SHA-256 of the oracle's output for
the synthetic A4 pages the benchmark processes.

TEST INFRASTRUCTURE: runs in the build container (oracle/_build/liboracle.so,
the C restatement of the reference CPU path, pinned to the reference goldens by
tests/test_oracle_golden.py).  The GPU side (tests/test_runner_gpu.py, __graft_entry__.smoke() and
bench.py's verification after the timed region) compares the HIP pipeline's
outputs with these hashes, so the exact benchmarked configuration is
parity-checked without running the oracle on the GPU box.

Pages: 0..999 (rank 0's whole 1000-page shard: the runner hands chunks to
whichever batch is idle, so which chunks stay resident after the timed passes
varies) and, for ranks 1..7 of a sharded run (1000 pages per rank), the first
16 pages of each shard.  Hashes already in the output file are kept.
Options: the reference defaults (uphip_options_init == lib/options.c).
Hash: SHA-256 over the output rows' visible bytes (GRAY8, W bytes per row).

C4 (--which c4 -> c4_hashes.json): RGB24 9920x7016 double-page sheets 0..15
(synth.h synth_rgb_channel) with unpaper_hip.workloads.c4_options (layout
double, bilinear deskew, border wipe); hash over the saved RGB24 rows.

usage: python3 tests/golden/make_bench_hashes.py [--threads N] [--which a4|c4]
"""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))

from oracle_py import Oracle  # noqa: E402
from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip.hostimage import HostImage  # noqa: E402
from unpaper_hip.pipeline import synth_page_host, synth_sheet_rgb_host  # noqa: E402
from unpaper_hip.workloads import C4_H, C4_W, c4_options  # noqa: E402

W, H = 2480, 3508


def page_list():
    pages = list(range(1000))
    for r in range(1, 8):
        pages += [r * 1000 + i for i in range(16)]
    return pages


def page_hash(oracle, opts, page):
    src = HostImage.from_array(synth_page_host(W, H, page), A.FMT_GRAY8)
    sheet, fmt, _ = oracle.process_sheet(opts, [src])
    out = oracle.convert_for_save(sheet, fmt)
    assert (out.width, out.height, out.format) == (W, H, A.FMT_GRAY8)
    return hashlib.sha256(out.payload().tobytes()).hexdigest()


def c4_hash(oracle, opts, sheet):
    src = HostImage.from_array(synth_sheet_rgb_host(C4_W, C4_H, sheet), A.FMT_RGB24)
    out_sheet, fmt, _ = oracle.process_sheet(opts, [src])
    out = oracle.convert_for_save(out_sheet, fmt)
    assert (out.width, out.height, out.format) == (C4_W, C4_H, A.FMT_RGB24)
    return hashlib.sha256(out.payload().tobytes()).hexdigest()


def main_c4(args):
    oracle = Oracle()
    opts = c4_options(oracle.default_options())
    res = {}
    t0 = time.time()

    todo = list(range(args.c4_sheets))
    lock = threading.Lock()

    def work():
        while True:
            with lock:
                if not todo:
                    return
                k = todo.pop(0)
            res[k] = c4_hash(oracle, opts, k)

    ts = [threading.Thread(target=work) for _ in range(min(args.threads, args.c4_sheets))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    doc = {
        "generator": "tests/golden/make_bench_hashes.py --which c4 (oracle/oracle.c, "
                     "unpaper_hip.workloads.c4_options)",
        "width": C4_W, "height": C4_H, "format": "RGB24",
        "hash": "sha256 of visible output rows",
        "sheets": {str(k): res[k] for k in sorted(res)},
    }
    out = os.path.join(HERE, "c4_hashes.json")
    with open(out, "w") as f:
        json.dump(doc, f, indent=0)
        f.write("\n")
    print("wrote %d C4 hashes to %s in %.0f s" % (len(res), out, time.time() - t0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=os.path.join(HERE, "bench_hashes.json"))
    ap.add_argument("--which", default="a4", choices=("a4", "c4"))
    ap.add_argument("--c4-sheets", type=int, default=16,
                    help="C4: hash sheets 0 .. N-1 (the bench's whole 16-sheet workload)")
    args = ap.parse_args()
    if args.which == "c4":
        return main_c4(args)
    oracle = Oracle()
    opts = oracle.default_options()
    res = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            res = {int(k): v for k, v in json.load(f)["pages"].items()}
    todo = [p for p in page_list() if p not in res]
    lock = threading.Lock()
    t0 = time.time()

    def work():
        while True:
            with lock:
                if not todo:
                    return
                p = todo.pop(0)
            h = page_hash(oracle, opts, p)
            with lock:
                res[p] = h
                if len(res) % 32 == 0:
                    print("%d pages, %.0f s" % (len(res), time.time() - t0), flush=True)

    ts = [threading.Thread(target=work) for _ in range(args.threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    doc = {
        "generator": "tests/golden/make_bench_hashes.py (oracle/oracle.c, default options)",
        "width": W, "height": H, "format": "GRAY8", "hash": "sha256 of visible output rows",
        "pages": {str(p): res[p] for p in sorted(res)},
    }
    with open(args.out, "w") as f:
        json.dump(doc, f, indent=0, sort_keys=False)
        f.write("\n")
    print("wrote %d hashes to %s in %.0f s" % (len(res), args.out, time.time() - t0))


if __name__ == "__main__":
    main()
