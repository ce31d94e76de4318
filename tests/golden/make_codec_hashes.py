#!/usr/bin/env python3
"""Generate tests/golden/codec_hashes.json: SHA-256 of the oracle's output for
the decoded inputs of bench.py's codec and PDF legs, so that every output
page of those legs is checked (bench.py --config jpeg / jp2 / pdf).

TEST INFRASTRUCTURE: runs in the build container (oracle/_build/liboracle.so,
the C restatement of the reference CPU path, pinned to the reference goldens
by tests/test_oracle_golden.py).

Keys:
  jpeg_q95: page i (0..63) = the synthetic A4 page i (synth.h, rank 0's
            first pages) saved by PIL as JPEG quality 95 and decoded by PIL
            (libjpeg-turbo; the GPU JPEG decode equals it byte for byte,
            tests/test_jpeg.py) -> default options -> oracle -> hash of the
            GRAY8 rows.  The inputs of --config jpeg and of the PDF JPEG leg.
  jbig2_50: page k (0..49) of the reference's benchmark_jbig2_50page.pdf,
            decoded by this repository's JBIG2 decoder (the jbig2dec peer;
            pinned by its own hashes, tests/test_pdf.py) -> oracle -> hash.
  (The lossless JPEG 2000 inputs decode to the synthetic pages themselves:
  their hashes are bench_hashes.json's.)

usage: python3 tests/golden/make_codec_hashes.py [--threads N]
"""
import argparse
import hashlib
import io
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))

from oracle_py import Oracle  # noqa: E402
from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip.hostimage import HostImage  # noqa: E402
from unpaper_hip.pipeline import synth_page_host  # noqa: E402

W, H = 2480, 3508
NJPEG = 64
JBIG2_PDF = os.path.join(HERE, "pdf", "benchmark_jbig2_50page.pdf")


def jpeg_q95_input(page):
    """The decoded pixels of bench.py's JPEG input `page` (PIL encode + decode)."""
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(synth_page_host(W, H, page)).save(b, "JPEG", quality=95)
    return np.asarray(Image.open(io.BytesIO(b.getvalue()))).copy()


def jbig2_input(k):
    from unpaper_hip import pdf as P
    return P.PdfDocument.open(JBIG2_PDF).read_page(k).data[:, :W].copy()


def out_hash(oracle, opts, px):
    sheet, fmt, _ = oracle.process_sheet(opts, [HostImage.from_array(px, A.FMT_GRAY8)])
    out = oracle.convert_for_save(sheet, fmt)
    assert (out.width, out.height, out.format) == (W, H, A.FMT_GRAY8)
    return hashlib.sha256(out.payload().tobytes()).hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    path = os.path.join(HERE, "codec_hashes.json")
    res = {"jpeg_q95": {}, "jbig2_50": {}}
    if os.path.exists(path):
        with open(path) as f:
            res.update({k: v for k, v in json.load(f).items() if isinstance(v, dict)})
    todo = [("jpeg_q95", i) for i in range(NJPEG) if str(i) not in res["jpeg_q95"]]
    todo += [("jbig2_50", k) for k in range(50) if str(k) not in res["jbig2_50"]]
    oracle = Oracle()
    opts = oracle.default_options()
    lock = threading.Lock()
    t0 = time.time()

    def work():
        while True:
            with lock:
                if not todo:
                    return
                key, i = todo.pop(0)
            px = jpeg_q95_input(i) if key == "jpeg_q95" else jbig2_input(i)
            h = out_hash(oracle, opts, px)
            with lock:
                res[key][str(i)] = h
                print("%s %d %s (%.0f s)" % (key, i, h[:12], time.time() - t0), flush=True)

    ts = [threading.Thread(target=work) for _ in range(args.threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for key in ("jpeg_q95", "jbig2_50"):
        res[key] = dict(sorted(res[key].items(), key=lambda kv: int(kv[0])))
    res["_doc"] = ("SHA-256 of the oracle's GRAY8 output rows for bench.py's codec/PDF inputs; "
                   "tests/golden/make_codec_hashes.py")
    with open(path, "w") as f:
        json.dump(res, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
