#!/usr/bin/env python3
"""PDF in -> cleaned PDF out on the GPU: the peer of the reference's
pdf_pipeline_batch_process (pdf/pdf_pipeline_batch.h; `unpaper in.pdf
out.pdf`), on the runner's PDF source and sink.

    python tools/pdf_pipeline.py in.pdf out.pdf [--pdf-quality fast|high]
        [--pdf-dpi N] [--jpeg-quality Q] [--input-pages 1|2] [--output-pages 1|2]

Every input page is decoded where its codec runs (JPEG / JPEG 2000 on the
device, JBIG2 / CCITT / Flate on the load pool), the sheets go through the
default pipeline, and each output page is encoded on the device (JPEG, or
lossless JPEG 2000 with --pdf-quality high) into one PDF with the input's
metadata.  Pages must share the first page's image geometry (the runner's
batches are of one page size); a page that does not is left out of the
output, as the reference's page accumulator leaves out failed pages.
--pdf-dpi 0 (the default here) takes the page images as they are; a dpi
applies the reference's size check (an image off the page size would need
a rasteriser and fails).
"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))

from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip import pdf as P  # noqa: E402
from unpaper_hip.device import load_library  # noqa: E402
from unpaper_hip.pipeline import Runner, sink_pdf, source_page_count, source_pdf  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("--pdf-quality", choices=("fast", "high"), default="fast")
    ap.add_argument("--pdf-dpi", type=int, default=0)
    ap.add_argument("--jpeg-quality", type=int, default=0, help="0 = 85 (PDF_OUTPUT_JPEG_QUALITY)")
    ap.add_argument("--input-pages", type=int, default=1, choices=(1, 2))
    ap.add_argument("--output-pages", type=int, default=1, choices=(1, 2))
    ap.add_argument("--sheets-per-batch", type=int, default=16)
    ap.add_argument("--streams", type=int, default=8)
    args = ap.parse_args()

    L = load_library()
    doc = P.PdfDocument.open(args.input)
    w, h, fmt = doc.page_probe(0, args.pdf_dpi)
    meta = doc.metadata()
    opts = A.Options()
    L.uphip_options_init(C.byref(opts))
    opts.input_count = args.input_pages
    opts.output_count = args.output_pages
    src = source_pdf(args.input, args.pdf_dpi)
    npages = source_page_count(src)
    jobs = npages // args.input_pages
    snk = sink_pdf(args.output, meta, args.pdf_dpi if args.pdf_dpi else 0, args.jpeg_quality,
                   1 if args.pdf_quality == "high" else 0)
    r = Runner(opts, args.sheets_per_batch, w, h, fmt, devices=(0,), streams=args.streams)
    try:
        t0 = time.perf_counter()
        failed, err = r.run_host(jobs, src, snk)
        snk.finish()
        dt = time.perf_counter() - t0
    finally:
        r.close()
    out = P.PdfDocument.open(args.output)
    print("%s: %d pages in, %d sheets, %d pages out, %d failed%s, %.2f s (%.1f sheets/s)"
          % (args.output, npages, jobs, out.page_count, failed, (" (" + err + ")") if failed else "",
             dt, jobs / dt if dt > 0 else 0.0))
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
