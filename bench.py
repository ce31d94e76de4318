#!/usr/bin/env python3
"""bench.py — pages/s of the per-sheet cleanup path on MI355X.

Workload (BASELINE.json configs[2], the metric's configuration): 1000
deterministic synthetic GRAY8 A4@300dpi pages (2480x3508)
per GPU, default unpaper options (the full sheet_process.c pipeline:
blackfilter, noisefilter, blurfilter, grayfilter, mask scan, deskew with
cubic rotation, mask centering, border scan), driven by the native runner
(uphip_runner_*, the lib/batch_worker.c peer): one host thread per device,
`--streams` batches of `--batch` sheets in flight per device.  The pages are
generated straight into HBM before the clock starts; `value` counts pages
processed with inputs and outputs resident in HBM (figure 1 of BASELINE.md
§3).  Figures 2 (+ H2D/D2H through pinned staging) and 3 (+ PNM write) are
measured after it with the host-fed runner over the same pages.

One step = one pass of the pipeline over every page of each device's shard.
N>1, driver style (torch.distributed.run): one process per GPU, pages sharded
by rank, no data-path collective; a gloo group only provides the barrier and
the max-over-ranks of the elapsed time.  N>1 without torchrun (`--gpus N`):
one process, one runner thread per device (the reference's thread pool bound
to devices), device d processing pages [d*P, (d+1)*P).

After the timed region every resident output page with a committed oracle
hash (tests/golden/bench_hashes.json, tests/golden/make_bench_hashes.py) is
hashed and compared; a mismatch fails the run.  A library built with the
timing diagnostics (make lib DIAG=1) or an UPHIP_DIAG_* variable is refused
unless --tuning (the line then says "valid": false).

Extra fields: `roofline` for the dominant kernel (the bicubic rotation),
timed with the HIP events its batch records on its own stream around the
launch; `cpu_baseline` = the oracle's restatement of the reference CPU path
on the host share of cores (rank 0, N=1 only); `latency_c2` = one A4 page
alone through the pipeline; `host_io` = figures 2 and 3; `c4` = BASELINE
configs[3] (16 RGB24 600 dpi double-page sheets, 4 per batch, 3 timed passes)
with its sheets/s, latency, bilinear-rotate roofline and every sheet checked
against tests/golden/c4_hashes.json (N=1 only; `--config c4` prints it alone).
"""
import argparse
import ctypes as C
import hashlib
import io
import json
import os
import shutil
import statistics
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))

# The HIP library is loaded before torch so that one HIP runtime (/opt/rocm)
# serves the process; torch is only used for torch.distributed (gloo).
from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip.device import load_library, UnpaperHipError  # noqa: E402
from unpaper_hip.pipeline import (Batch, DeviceBuffer, Runner, sink_discard,  # noqa: E402
                                  sink_jp2, sink_jpeg, sink_memory, sink_pnm, source_memory,
                                  source_pnm)
from unpaper_hip.workloads import A4_H, A4_W, C4_H, C4_W, c4_options  # noqa: E402

METRIC = "pages/sec + Mpixel/s, 1000-page GRAY8 A4@300dpi batch, 1/2/4/8 GPU"
W, H = A4_W, A4_H
HBM_PEAK_GBS = 8000.0                   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
ALG_BYTES_PER_PAGE = 10 * W * H         # SURVEY.md §8(d) fixed credit (86 998 400 B)
GOLDEN = os.path.join(ROOT, "tests", "golden")
NDISTINCT = 64                          # distinct input files of the codec / PDF legs

# Algorithmic HBM bytes per page of each timed stage (DESIGN.md "Kernels"):
# the bytes the stage must move at minimum, in units of one W*H plane.
STAGE_PLANES = {
    "decode": 2.0,          # page -> sheet plane (read + write)
    "noisefilter": 1.0,     # classify reads the plane once
    "blurfilter": 1.0,      # block counts read the plane once
    "grayfilter": 1.0,      # tile sums read the plane once
    "masks_deskew": 1.0,    # column sums over the plane
    "deskew_rotate": 2.0,   # rotated gather read + write
    "masks_center": 1.0,    # column sums over the plane
    "center": 2.0,          # mask move read + write
}
ROOFLINE_STAGE = "deskew_rotate"
ROOFLINE_KERNEL = {"c3": "k_rotate_cubic_g8f",
                   "c4": "k_rotate_lin<F_RGB24> (bilinear, both masks of a sheet in one launch)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=("c3", "c4", "jpeg", "jp2", "pdf"),
                    help="c3: BASELINE configs[2] (the metric); c4: configs[3], RGB24 600dpi "
                         "double-page sheets, layout double, bilinear, border wipe; jpeg: the "
                         "JPEG decode peer (SURVEY f3) feeding the runner from JPEG files")
    ap.add_argument("--pages", type=int, default=0,
                    help="pages (c3) / sheets (c4) per GPU (default 1000 / 16)")
    ap.add_argument("--batch", type=int, default=0, help="sheets per batch (default 64 / 4)")
    ap.add_argument("--streams", type=int, default=16, help="batches (HIP streams) per device")
    ap.add_argument("--hw-queues", type=int, default=24,
                    help="GPU_MAX_HW_QUEUES for this process (HIP default 4, at most 32)")
    ap.add_argument("--cpu-pages", type=int, default=0,
                    help="CPU baseline sample (0 = 8 pages per host thread)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the host share: OMP_NUM_THREADS, else os.cpu_count()")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-host-io", action="store_true", help="skip figures 2 and 3")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the C2 single-page latency and the C4 single-sheet runs")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the C4 object of the default line (16 RGB24 sheets, verified)")
    ap.add_argument("--codec-streams", type=int, default=0,
                    help="batches in flight for --config jpeg / jp2 (0 = 8 / 16)")
    ap.add_argument("--c4-streams", type=int, default=0,
                    help="C4 batches (HIP streams) in flight (0 = --streams)")
    ap.add_argument("--host-batch", type=int, default=32, help="sheets per batch, host-fed runs")
    ap.add_argument("--host-streams", type=int, default=8, help="batches per device, host-fed")
    ap.add_argument("--valu", default=os.path.join(ROOT, "profiles", "valu.json"),
                    help="per-kernel VALU instructions per sheet (profiles/clock_table.py)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC HBM bytes per launch / per page from rocprofv3 --pmc passes")
    ap.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--probe", type=int, default=3,
                    help="isolated single-stream launches after the timed region that time "
                         "the roofline kernel (0 = use the concurrent timed-region spans)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the oracle-hash check of the resident outputs")
    ap.add_argument("--tuning", action="store_true",
                    help="allow a diagnostics build / UPHIP_DIAG_* (the line is marked invalid)")
    return ap.parse_args()


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def _reduce(self, v, op):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return float(t.item())

    def max(self, v):
        return self._reduce(v, "MAX")

    def sum(self, v):
        return self._reduce(v, "SUM")

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def shard_plan(world, rank, local_rank, ngpus_flag, ndev, pages):
    """(devices this process drives, first global page of each, n_gpus of the job)."""
    if world > 1:
        return [local_rank % max(ndev, 1)], [rank * pages], world
    if ngpus_flag > ndev:
        raise UnpaperHipError("--gpus %d but only %d HIP devices" % (ngpus_flag, ndev))
    return list(range(ngpus_flag)), [i * pages for i in range(ngpus_flag)], ngpus_flag


def diag_guard(version, environ, tuning):
    """Refuse timing-diagnostics builds and switches (they skip or repeat work).
    Returns whether the measurement is valid."""
    env = sorted(k for k in environ if k.startswith("UPHIP_DIAG"))
    bad = ("diag" in version) or bool(env)
    if bad and not tuning:
        raise SystemExit("bench.py: refusing to time a diagnostics build or UPHIP_DIAG_* (%s; %s); "
                         "use `make lib` without DIAG and unset the variables" % (version, env))
    return not bad


def load_hashes(name, key):
    try:
        with open(os.path.join(GOLDEN, name)) as f:
            return json.load(f).get(key, {})
    except (OSError, ValueError):
        return {}


def note(msg):
    """A progress line on stderr (long legs print one a phase, so a watcher
    sees the run alive)."""
    print("bench.py: %s" % msg, file=sys.stderr, flush=True)


def sha_rows(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def pmap(fn, items, threads):
    """fn over items on a thread pool (hashlib, PIL and numpy release the GIL
    on large buffers); results in order."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max(1, min(16, threads))) as ex:
        return list(ex.map(fn, items))


def verify_resident(runner, devices, firsts, npages, bsz, hashes):
    """Hash every resident output page that has a committed oracle hash: each
    batch holds the outputs of the last chunk it ran (uphip_runner_slot_chunk;
    the runner hands chunks to whichever batch is idle)."""
    checked = bad = 0
    for i in range(len(devices)):
        for k in range(runner.streams):
            ch = runner.slot_chunk(i, k)
            if ch is None:
                continue
            first, n = ch
            b = runner.batch(i, k)
            for s in range(n):
                g = str(firsts[i] + first + s)
                if g not in hashes:
                    continue
                out = b.output(s)
                checked += 1
                if hashlib.sha256(out.payload().tobytes()).hexdigest() != hashes[g]:
                    bad += 1
                    print("bench: page %s differs from the oracle (device %d batch %d sheet %d)"
                          % (g, devices[i], k, s), file=sys.stderr)
    return checked, bad


def stage_totals(runner, ndev):
    totals = {}
    for i in range(ndev):
        for k in range(runner.streams):
            for name, ms in runner.batch(i, k).stage_times():
                totals[name] = totals.get(name, 0.0) + ms
    return totals


def probe_kernel(runner, shard, n0, stage, count):
    """Isolated launches of one batch on one stream, the GPU otherwise idle."""
    b = runner.batch(0, 0)
    out = []
    for _ in range(count):
        b.run_device(n0, shard[0], shard[1], shard[2])
        b.wait()
        out.append(sum(ms for name, ms in b.stage_times() if name == stage))
    return out


def valu_frac_of(path, kernel, units, avg_ms):
    """VALU-issue fraction of one launch of `units` sheets lasting avg_ms:
    committed VALU instructions per sheet x 4 cycles / (1024 SIMDs x clock x
    time), the clock being the one measured in the same PMC run."""
    try:
        with open(path) as f:
            ks = json.load(f)["kernels"]
        # the one-tile-per-block instantiation (<false>) is the full-batch launch
        k = ks[kernel] if kernel in ks else ks[kernel + "<false>"]
    except (OSError, ValueError, KeyError):
        return None
    if avg_ms <= 0:
        return None
    return round(k["valu_insts_per_sheet"] * units * 4 / (1024 * k["clock_ghz"] * 1e9 * avg_ms * 1e-3), 4)


def c4_traffic(path):
    """HBM bytes per sheet of the C4 rotate (FETCH_SIZE x2 + WRITE_SIZE,
    tools/traffic_c4.sh), the same unit as its alg_bytes_per_launch."""
    try:
        with open(path) as f:
            return json.load(f).get("c4", {}).get("hbm_bytes_per_sheet")
    except (OSError, ValueError):
        return None


def traffic_of(path, key, units):
    try:
        with open(path) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None, None
    per_page = doc.get("bytes_per_page", {}).get(key)
    return (int(per_page * units) if per_page else None), doc.get("pipeline_bytes_per_page")


def device_pages_to_host(L, pages, pitch, stride, npages, w, h, bpp=1):
    """Copy device-resident pages into a dense host array (outside any clock)."""
    out = np.empty((npages, h, w * bpp), np.uint8)
    tmp = np.empty((h, pitch), np.uint8)
    for p in range(npages):
        if L.uphip_memcpy_dtoh(tmp.ctypes.data, pages.ptr + p * stride, pitch * h) != 0:
            raise UnpaperHipError("memcpy_dtoh failed")
        out[p] = tmp[:, :w * bpp]
    return out


def latency_c2(L, opts, page_host, pages_ptr, pitch, stride, reps=7):
    """C2 (BASELINE configs[1]): one A4 page alone through the full pipeline
    on an idle GPU, median of `reps` runs after one warm-up: input resident
    in HBM, and with the host copies (set_input + run + get_output)."""
    b = Batch(opts, 1, W, H, A.FMT_GRAY8)
    try:
        dev, host = [], []
        for r in range(reps + 1):
            t0 = time.perf_counter()
            b.run_device(1, pages_ptr, pitch, stride)
            b.wait()
            if r:
                dev.append((time.perf_counter() - t0) * 1e3)
        # where a lone page's time goes: one more run with stage events
        b.set_timing(True)
        b.run_device(1, pages_ptr, pitch, stride)
        b.wait()
        stages = {k: round(v, 3) for k, v in b.stage_times()}
        b.set_timing(False)
        for r in range(reps + 1):
            t0 = time.perf_counter()
            if L.uphip_batch_set_input(b.handle, 0, page_host.ctypes.data, W) != 0:
                raise UnpaperHipError("set_input failed")
            b.run(1)
            b.wait()
            b.output(0)
            if r:
                host.append((time.perf_counter() - t0) * 1e3)
        return round(statistics.median(dev), 3), round(statistics.median(host), 3), stages
    finally:
        b.close()


def host_io(opts, dev0, host_in, npages, args, threads):
    """Figures 2 and 3 of BASELINE.md §3 on device `dev0`: the pages fed from
    host RAM through pinned staging (H2D), processed, brought back (D2H) into
    host RAM; then the same with the sheets written as PGM files (the encode
    queue) into a tmpfs directory.  One untimed warm-up pass each."""
    out = {}
    r = Runner(opts, args.host_batch, W, H, A.FMT_GRAY8, devices=(dev0,),
               streams=args.host_streams, host_threads=threads)
    try:
        host_out = np.empty((npages, H, r.out_linesize), np.uint8)
        src = source_memory(host_in.ctypes.data, W, W * H, npages, keep=host_in)
        snk = sink_memory(host_out.ctypes.data, r.out_linesize, r.out_linesize * H, npages,
                          keep=host_out)
        for rep in range(2):
            t0 = time.perf_counter()
            failed, err = r.run_host(npages, src, snk)
            t = time.perf_counter() - t0
            if failed:
                raise UnpaperHipError("host-fed run: %d failed: %s" % (failed, err))
        st = r.stats()
        # every page of the timed pass against the oracle's hashes
        hashes = load_hashes("bench_hashes.json", "pages")
        sample = [p for p in range(npages) if str(p) in hashes]
        got = pmap(lambda p: sha_rows(host_out[p][:, :W]), sample, threads)
        bad = sum(g != hashes[str(p)] for g, p in zip(got, sample))
        if bad:
            raise SystemExit("bench.py: host-fed outputs differ from the oracle (%d of %d)"
                             % (bad, len(sample)))
        out["h2d_d2h"] = {"value": round(npages / t, 2), "unit": "pages/s",
                          "load_s": round(st.load_s, 3), "store_s": round(st.store_s, 3),
                          "verified": len(sample)}
        del snk
        verified_pages = set(sample)

        def per_chunk_check(snk, n, check):
            """Re-run the first n pages in chunks of 64 (file names wrap every
            64 pages, so after a chunk file i holds page k + i) and check
            every file; untimed, after the timed passes."""
            done = 0
            for k in range(0, n, 64):
                m = min(64, n - k)
                src_k = source_memory(host_in[k:].ctypes.data, W, W * H, m, keep=host_in)
                failed, err = r.run_host(m, src_k, snk)
                if failed:
                    raise UnpaperHipError("check run: %d failed: %s" % (failed, err))
                done += sum(pmap(lambda i: check(k + i, i), range(m), threads))
            return done
        tmpdir = tempfile.mkdtemp(prefix="uphip_bench_",
                                  dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        try:
            snk = sink_pnm(os.path.join(tmpdir, "out_%04lld.pgm"), 64)
            for rep in range(2):
                t0 = time.perf_counter()
                failed, err = r.run_host(npages, src, snk)
                t = time.perf_counter() - t0
                if failed:
                    raise UnpaperHipError("PNM run: %d failed: %s" % (failed, err))
            st = r.stats()
            note("host-fed: PNM written; JPEG sink")
            out["pnm_write"] = {"value": round(npages / t, 2), "unit": "pages/s",
                                "load_s": round(st.load_s, 3), "store_s": round(st.store_s, 3),
                                "files": "PGM (P5) into tmpfs, 64 names reused"}
            # the GPU JPEG output branch (sheet_stages.c:554-581): pages encoded
            # on the device after their batch, only the files cross PCIe
            snk = sink_jpeg(os.path.join(tmpdir, "out_%04lld.jpg"), 64, 85, 0)
            for rep in range(2):
                t0 = time.perf_counter()
                failed, err = r.run_host(npages, src, snk)
                t = time.perf_counter() - t0
                if failed:
                    raise UnpaperHipError("JPEG run: %d failed: %s" % (failed, err))
            st = r.stats()
            # every page's file equals libjpeg-turbo's (PIL) encode of that
            # page's oracle-verified sheet
            from PIL import Image

            def jpeg_same(p, i):
                if p not in verified_pages:
                    return 0
                b = io.BytesIO()
                Image.fromarray(np.ascontiguousarray(host_out[p][:, :W])).save(b, "JPEG", quality=85)
                with open(os.path.join(tmpdir, "out_%04d.jpg" % i), "rb") as f:
                    return int(f.read() == b.getvalue())
            same = per_chunk_check(snk, npages, jpeg_same)
            if same != len([p for p in range(npages) if p in verified_pages]):
                raise SystemExit("bench.py: JPEG files differ from PIL's encode of the sheets")
            kb = os.path.getsize(os.path.join(tmpdir, "out_0000.jpg")) / 1e3
            out["jpeg_write"] = {"value": round(npages / t, 2), "unit": "pages/s",
                                 "load_s": round(st.load_s, 3), "store_s": round(st.store_s, 3),
                                 "files": "JPEG q85 (GPU encode) into tmpfs, 64 names reused, "
                                          "%.0f kB a page" % kb,
                                 "verified": same}
            # the lossless JPEG 2000 output branch (encode_queue.c:883-962):
            # transforms and code-blocks on the device per output page (the
            # store tasks), packets on the host; files decode (PIL) to the
            # oracle-verified sheets
            note("host-fed: JPEG files checked (%d); JP2 sink" % same)
            nj = min(npages, 256)
            snk = sink_jp2(os.path.join(tmpdir, "out_%04lld.jp2"), 64)
            for rep in range(2):
                t0 = time.perf_counter()
                failed, err = r.run_host(nj, src, snk)
                t = time.perf_counter() - t0
                if failed:
                    raise UnpaperHipError("JP2 run: %d failed: %s" % (failed, err))
            st = r.stats()

            def jp2_same(p, i):  # every file decodes (OpenJPEG) to its verified sheet
                if p not in verified_pages:
                    return 0
                back = np.asarray(Image.open(os.path.join(tmpdir, "out_%04d.jp2" % i)))
                return int(np.array_equal(back, host_out[p][:, :W]))
            same = per_chunk_check(snk, nj, jp2_same)
            if same != len([p for p in range(nj) if p in verified_pages]):
                raise SystemExit("bench.py: JP2 files do not decode to the sheets")
            kb = os.path.getsize(os.path.join(tmpdir, "out_0000.jp2")) / 1e3
            out["jp2_write"] = {"value": round(nj / t, 2), "unit": "pages/s",
                                "load_s": round(st.load_s, 3), "store_s": round(st.store_s, 3),
                                "files": "lossless JP2 (GPU transforms + code-blocks) into tmpfs, "
                                         "%d pages, 64 names reused, %.0f kB a page" % (nj, kb),
                                "verified": same}
        finally:
            shutil.rmtree(tmpdir, ignore_errors=True)
            del host_out
        out["config"] = {"sheets_per_batch": args.host_batch, "streams": args.host_streams,
                         "host_threads": threads, "staging": "pinned, per batch, in + out",
                         "source": "pages in host RAM (decoded)"}
    finally:
        r.close()
    return out


def cpu_baseline(host_pages, npages, threads):
    """The oracle (C restatement of the reference --device=cpu path), one page
    per thread at a time; ctypes releases the GIL inside the C call."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_py import Oracle
    from unpaper_hip.hostimage import HostImage
    oracle = Oracle()
    opts = oracle.default_options()
    imgs = [HostImage.from_array(host_pages[p], A.FMT_GRAY8) for p in range(npages)]
    nxt = [0]
    lock = threading.Lock()

    def work():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= npages:
                return
            oracle.process_sheet(opts, [imgs[i]])

    ts = [threading.Thread(target=work) for _ in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return npages / (time.perf_counter() - t0)


def host_threads_share():
    """Host threads this job may use: the box sets OMP_NUM_THREADS to the
    GPU's CPU share (os.cpu_count() reports the whole machine there)."""
    v = os.environ.get("OMP_NUM_THREADS")
    try:
        return max(1, int(v)) if v else (os.cpu_count() or 1)
    except ValueError:
        return os.cpu_count() or 1


def run_jpeg(args, L, d, devices, firsts, n_gpus, version, valid, codec="jpeg"):
    """The JPEG decode peer in the runner: synthetic A4 GRAY8
    pages saved by PIL as JPEG quality 95 (tmpfs), read by a runner file
    source (marker parse + unstuffing on the load pool into pinned memory;
    Huffman decode of every page of a chunk in one set of launches, then the
    IDCT into the batch's input slots, on the device), the default pipeline,
    sheets discarded.  PCIe- and host-inclusive: a figure of its own, never `value`
    of the C3 line.  64 distinct input files; the sheets come back into host
    RAM and every page is checked against the oracle's hash of its decoded
    input (tests/golden/codec_hashes.json for JPEG, bench_hashes.json for the
    lossless JPEG 2000 files).  codec "jp2": the same pages saved
    losslessly as JPEG 2000 (OpenJPEG's defaults), headers and packet headers
    parsed on the load pool, every code-block of a chunk decoded on the
    device in one launch, then the wavelet into the input slots."""
    from PIL import Image
    from concurrent.futures import ThreadPoolExecutor
    n = args.pages or 512
    threads = host_threads_share()
    tmpdir = tempfile.mkdtemp(prefix="uphip_jpeg_",
                              dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        # 64 distinct pages, reused round robin (the decode cost does not
        # depend on the name)
        def make(i):
            g = np.empty((H, W), np.uint8)
            L.uphip_synth_page_host(g.ctypes.data, W, W, H, firsts[0] + i)
            if codec == "jp2":
                path = os.path.join(tmpdir, "p%02d.jp2" % i)
                Image.fromarray(g).save(path, "JPEG2000")
            else:
                path = os.path.join(tmpdir, "p%02d.jpg" % i)
                Image.fromarray(g).save(path, "JPEG", quality=95)
            return path
        with ThreadPoolExecutor(min(16, threads)) as ex:
            uniq = list(ex.map(make, range(NDISTINCT)))
        paths = [uniq[i % NDISTINCT] for i in range(n)]
        mb = sum(os.path.getsize(p) for p in uniq) / NDISTINCT / 1e6
        opts = A.Options()
        L.uphip_options_init(C.byref(opts))
        # batches in flight: JPEG 2000 chunks wait on their one code-block
        # launch, so more of them in flight pay (tools/codec_streams.sh: 32 x 8
        # 698, 32 x 16 856, 64 x 8 797, 64 x 16 821 pages/s); JPEG is host-bound
        streams = args.codec_streams or (16 if codec == "jp2" else 8)
        r = Runner(opts, args.host_batch, W, H, A.FMT_GRAY8, devices=devices[:1], streams=streams,
                   host_threads=threads)
        try:
            src = source_pnm(paths)
            for rep in range(2):  # one warm-up pass (pinned buffers grow once)
                t0 = time.perf_counter()
                failed, err = r.run_host(n, src, sink_discard())
                t = time.perf_counter() - t0
                if failed:
                    raise UnpaperHipError("%s run: %d failed: %s" % (codec, failed, err))
            st = r.stats()
            # then the same pages once more (untimed) with the sheets brought
            # back into host RAM (registered, DMA'd straight into place): every
            # page is hashed below.  The timed pass discards its sheets, as
            # the figure of earlier rounds did (a D2H of every sheet costs the
            # file-fed rate ~20 % on the shared link).
            host_out = np.empty((n, H, r.out_linesize), np.uint8)
            snk = sink_memory(host_out.ctypes.data, r.out_linesize, r.out_linesize * H, n,
                              keep=host_out)
            if not args.no_verify:
                failed, err = r.run_host(n, src, snk)
                if failed:
                    raise UnpaperHipError("%s check run: %d failed: %s" % (codec, failed, err))
        finally:
            r.close()
        checked = 0
        if not args.no_verify:
            # the oracle's hashes of the decoded inputs' cleaned sheets: JPEG
            # from tests/golden/codec_hashes.json (PIL's decode of the same
            # files), lossless JPEG 2000 = the synthetic pages themselves
            if codec == "jp2":
                hs = load_hashes("bench_hashes.json", "pages")
                exp = [hs[str(firsts[0] + i)] for i in range(NDISTINCT)]
            else:
                if firsts[0] != 0:
                    raise SystemExit("bench.py: JPEG hashes exist for rank 0's pages only")
                hs = load_hashes("codec_hashes.json", "jpeg_q95")
                exp = [hs[str(i)] for i in range(NDISTINCT)]
            got = pmap(lambda i: sha_rows(host_out[i][:, :W]), range(n), threads)
            bad = [i for i in range(n) if got[i] != exp[i % NDISTINCT]]
            if bad:
                raise SystemExit("bench.py: %s pages %s differ from the oracle" % (codec, bad[:8]))
            checked = n
        del host_out, snk
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    what = ("JPEG 2000 files through the runner (JPEG 2000 decode peer)" if codec == "jp2" else
            "JPEG files through the runner (JPEG decode peer)")
    made = "PIL JPEG 2000 lossless" if codec == "jp2" else "PIL JPEG quality 95"
    return {"metric": "pages/s, A4 GRAY8 " + what,
            "value": round(n / t, 2), "unit": "pages/s", "n_gpus": 1, "higher_is_better": True,
            "dtype": "u8", "data": "synthetic (%s, %.2f MB a page)" % (made, mb),
            "host_threads": threads, "load_s": round(st.load_s, 3),
            "config": {"pages": n, "sheets_per_batch": args.host_batch, "streams": streams,
                       "source": "%s files in tmpfs (%d distinct, round robin)"
                                 % (codec.upper(), NDISTINCT),
                       "sink": "discarded (timed); every page then re-run into host RAM and "
                               "hashed (untimed)"},
            "verified": checked, "library": version, "valid": valid}


def run_pdf(args, L, d, devices, firsts, n_gpus, version, valid):
    """The PDF pipeline (pdf/pdf_pipeline_cpu_batch.c; SURVEY §8 f rank 4):
    PDF in -> pages decoded (JBIG2 on the load pool, JPEG on the device) ->
    the default pipeline -> every sheet JPEG-encoded on the device into one
    PDF (--pdf-quality fast, 300 dpi).  Two legs:
      * the reference's own benchmark file (tools/bench_jbig2_pdf.py):
        tests/golden/pdf/benchmark_jbig2_50page.pdf, 50 A4 pages of JBIG2
        generic regions;
      * a PDF of 512 A4 JPEG pages (quality 95) written by our writer.
    File-to-file, host-inclusive: figures of their own, never `value` of the
    C3 line.  Every page of each leg is checked: the sheets of an untimed
    pass against the oracle's hashes of the decoded pages (our JBIG2 decode /
    PIL's JPEG decode, tests/golden/codec_hashes.json), and every page of the
    timed pass's output PDF against PIL's quality-85 encode of its sheet."""
    from PIL import Image
    from concurrent.futures import ThreadPoolExecutor
    from unpaper_hip import pdf as P
    from unpaper_hip.pipeline import sink_pdf, source_pdf, source_page_count
    threads = host_threads_share()
    tmpdir = tempfile.mkdtemp(prefix="uphip_pdf_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    legs = {}
    try:
        jb = os.path.join(ROOT, "tests", "golden", "pdf", "benchmark_jbig2_50page.pdf")
        jpg_pdf = os.path.join(tmpdir, "jpeg512.pdf")
        n_jpeg = args.pages or 512

        def make(i):
            g = np.empty((H, W), np.uint8)
            L.uphip_synth_page_host(g.ctypes.data, W, W, H, firsts[0] + i)
            b = io.BytesIO()
            Image.fromarray(g).save(b, "JPEG", quality=95)
            return b.getvalue()
        with ThreadPoolExecutor(min(16, threads)) as ex:
            uniq = list(ex.map(make, range(NDISTINCT)))
        w = P.PdfWriter.create(jpg_pdf, {"title": "bench"}, 300)
        for i in range(n_jpeg):
            w.add_page_jpeg(uniq[i % NDISTINCT], W, H)
        w.close()
        opts = A.Options()
        L.uphip_options_init(C.byref(opts))
        pdf_streams = args.codec_streams or 8
        r = Runner(opts, args.host_batch, W, H, A.FMT_GRAY8, devices=devices[:1], streams=pdf_streams,
                   host_threads=threads)
        try:
            for name, path in (("jbig2_50", jb), ("jpeg_%d" % n_jpeg, jpg_pdf)):
                src = source_pdf(path, 300)
                n = source_page_count(src)
                meta = P.PdfDocument.open(path).metadata()
                out = os.path.join(tmpdir, "out_%s.pdf" % name)
                best = None
                for rep in range(3):  # the first pass warms the pinned buffers
                    k = sink_pdf(out, meta, 300, 0, 0)
                    t0 = time.perf_counter()
                    failed, err = r.run_host(n, src, k)
                    k.finish()
                    t = time.perf_counter() - t0
                    k.close()
                    if failed:
                        raise UnpaperHipError("pdf %s: %d failed: %s" % (name, failed, err))
                    if rep:
                        best = t if best is None else min(best, t)
                st = r.stats()
                d_out = P.PdfDocument.open(out)
                if d_out.page_count != n:
                    raise SystemExit("bench.py: pdf %s wrote %d pages of %d" % (name, d_out.page_count, n))
                checked = 0
                if not args.no_verify:
                    # every page: (1) an untimed pass into host RAM, each sheet
                    # against the oracle's hash of its decoded input
                    # (tests/golden/codec_hashes.json: our JBIG2 decode /
                    # PIL's JPEG decode); (2) every JPEG page of the timed
                    # pass's output PDF equals PIL's (libjpeg-turbo) quality-85
                    # encode of its verified sheet
                    if name == "jbig2_50":
                        hs = load_hashes("codec_hashes.json", "jbig2_50")
                        exp = [hs[str(i)] for i in range(n)]
                    else:
                        hs = load_hashes("codec_hashes.json", "jpeg_q95")
                        exp = [hs[str(i % NDISTINCT)] for i in range(n)]
                    host_out = np.empty((n, H, r.out_linesize), np.uint8)
                    snk = sink_memory(host_out.ctypes.data, r.out_linesize, r.out_linesize * H, n,
                                      keep=host_out)
                    failed, err = r.run_host(n, src, snk)
                    if failed:
                        raise UnpaperHipError("pdf %s check run: %s" % (name, err))
                    got = pmap(lambda i: sha_rows(host_out[i][:, :W]), range(n), threads)
                    bad = [i for i in range(n) if got[i] != exp[i]]
                    if bad:
                        raise SystemExit("bench.py: pdf %s pages %s differ from the oracle" % (name, bad[:8]))

                    tls = threading.local()

                    def page_same(i):
                        b = io.BytesIO()
                        Image.fromarray(np.ascontiguousarray(host_out[i][:, :W])).save(b, "JPEG", quality=85)
                        if not hasattr(tls, "doc"):
                            tls.doc = P.PdfDocument.open(out)
                        im = tls.doc.extract_page_image(i)
                        return int(im.format == P.IMAGE_JPEG and bytes(im.data) == b.getvalue())
                    same = sum(pmap(page_same, range(n), threads))
                    if same != n:
                        raise SystemExit("bench.py: pdf %s: %d of %d output pages differ from PIL's "
                                         "encode of the verified sheets" % (name, n - same, n))
                    checked = n
                    del host_out, snk
                legs[name] = {"pages": n, "pages_per_s": round(n / best, 2), "s": round(best, 3),
                              "load_s": round(st.load_s, 3), "store_s": round(st.store_s, 3),
                              "in_mb": round(os.path.getsize(path) / 1e6, 3),
                              "out_mb": round(os.path.getsize(out) / 1e6, 3), "verified": checked}
        finally:
            r.close()
    finally:
        shutil.rmtree(tmpdir, ignore_errors=True)
    return {"metric": "pages/s, A4 GRAY8 PDF -> PDF (JBIG2 or JPEG pages in, JPEG pages out)",
            "value": legs["jbig2_50"]["pages_per_s"], "unit": "pages/s", "n_gpus": 1,
            "higher_is_better": True, "dtype": "u8",
            "data": "the reference's benchmark_jbig2_50page.pdf; synthetic JPEG pages (PIL quality 95)",
            "host_threads": threads, "legs": legs,
            "config": {"sheets_per_batch": args.host_batch, "streams": args.codec_streams or 8, "dpi": 300,
                       "pdf_quality": "fast (JPEG 85)"},
            "library": version, "valid": valid}


def run_c4(args, L, d, devices, firsts, n_gpus, version, valid, nsheets=0, steps=0, warmup=-1,
           batch=0):
    """BASELINE configs[3]: RGB24 600dpi double-page sheets, layout double,
    bilinear deskew, border wipe; sheets/s and single-sheet latency.  Returns
    the C4 line (printed by `--config c4`, embedded as "c4" in the default
    line); every resident output sheet is checked against c4_hashes.json."""
    nsheets = nsheets or args.pages or 16
    steps = steps or args.steps
    warmup = args.warmup if warmup < 0 else warmup
    bsz = max(1, min(batch or args.batch or 4, nsheets))
    opts = A.Options()
    L.uphip_options_init(C.byref(opts))
    c4_options(opts)
    pitch = (3 * C4_W + 255) // 256 * 256
    stride = pitch * C4_H
    L.uphip_set_device(devices[0])
    pages = DeviceBuffer(stride * nsheets)
    if L.uphip_synth_sheets_rgb(pages.ptr, pitch, stride, C4_W, C4_H, firsts[0], nsheets) != 0:
        raise UnpaperHipError("synth_sheets_rgb failed")
    # batches in flight (--streams, as C3): more than a pass's chunks, so the
    # next pass's chunks start while a pass's flood-heavy chunk still runs on
    # its own batch -- a long job of C4 sheets keeps as many in flight
    # (tools/c4_streams.sh: 4 -> 316, 8 -> 439, 12 -> 476, 16 -> 494 sheets/s,
    # every resident sheet checked)
    streams = args.c4_streams or args.streams
    r = Runner(opts, bsz, C4_W, C4_H, A.FMT_RGB24, devices=devices[:1], streams=streams,
               timing=True)
    shard = [(pages.ptr, pitch, stride, nsheets)]
    if warmup:
        r.run_device(shard, passes=warmup)
    stage_totals(r, 1)
    d.barrier()
    t0 = time.perf_counter()
    failed, err = r.run_device(shard, passes=steps)
    d.barrier()
    elapsed = d.max(time.perf_counter() - t0)
    if failed:
        raise UnpaperHipError("c4 run: %s" % err)
    totals = stage_totals(r, 1)
    checked = bad = 0
    if not args.no_verify:
        checked, bad = verify_resident(r, devices[:1], firsts, nsheets, bsz,
                                       load_hashes("c4_hashes.json", "sheets"))
    r.close()
    # one sheet alone on an idle GPU: latency and the rotate launch (sheet 0,
    # no band), then every sheet once alone: the odd sheets carry the dark
    # band the blackfilter floods, and the heaviest one sets a batch's step
    lat, rot, lat_stages, per_sheet, heavy = [], [], {}, [], (None, -1.0, {})
    if not args.no_latency:
        b1 = Batch(opts, 1, C4_W, C4_H, A.FMT_RGB24, timing=True)
        try:
            for rep in range(4):
                t1 = time.perf_counter()
                b1.run_device(1, pages.ptr, pitch, stride)
                b1.wait()
                t2 = time.perf_counter()
                st = dict(b1.stage_times())
                if rep:
                    lat.append((t2 - t1) * 1e3)
                    rot.append(st.get(ROOFLINE_STAGE, 0.0))
                    lat_stages = st
            for sheet in range(nsheets):
                t1 = time.perf_counter()
                b1.run_device(1, pages.ptr + sheet * stride, pitch, stride)
                b1.wait()
                ms = (time.perf_counter() - t1) * 1e3
                st = dict(b1.stage_times())
                per_sheet.append(round(ms, 2))
                if ms > heavy[1]:
                    heavy = (sheet, ms, st)
        finally:
            b1.close()
    pages.close()
    alg_sheet = 10 * C4_W * C4_H * 3
    rot_alg = 2 * C4_W * C4_H * 3
    sheets_s = nsheets * steps * n_gpus / elapsed
    rot_ms = statistics.median(rot) if rot else 0.0
    ach = rot_alg / (rot_ms * 1e-3) / 1e9 if rot_ms else None
    line = {
            "metric": "sheets/s and per-sheet latency, RGB24 600dpi double-page scan (C4)",
            "value": round(sheets_s, 3), "unit": "sheets/s", "n_gpus": n_gpus,
            "steps": steps, "warmup": warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "latency_ms": round(statistics.median(lat), 2) if lat else None,
            "latency_of": "sheet 0 alone (no dark band)",
            "latency_stages_ms": {k: round(v, 3) for k, v in lat_stages.items()},
            "latency_band_ms": round(heavy[1], 2) if heavy[0] is not None else None,
            "latency_band_of": "the slowest sheet alone (sheet %s; odd sheets carry a 40-px dark "
                               "band the blackfilter floods)" % heavy[0],
            "latency_band_stages_ms": {k: round(v, 3) for k, v in heavy[2].items()},
            "latency_per_sheet_ms": per_sheet,
            "config": {"workload": "%d synthetic RGB24 9920x7016 double-page sheets per GPU, "
                                   "layout double, interpolate linear, border 60" % nsheets,
                       "sheets_per_batch": bsz, "streams": streams},
            "roofline": {"bound": "hbm", "kernel": ROOFLINE_KERNEL["c4"],
                         "achieved": round(ach, 1) if ach else None, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                         "traffic": c4_traffic(args.traffic), "avg_launch_ms": round(rot_ms, 3),
                         "launch_ms_from": "3 single-sheet runs, idle GPU (the deskew_rotate "
                                           "stage: the two-mask launch + the launch for sheets "
                                           "whose mask 1 depends on deskew 0)",
                         "alg_bytes_per_launch": rot_alg,
                         "pipeline_alg_bytes_per_sheet": alg_sheet,
                         "pipeline_frac": round(sheets_s / n_gpus * alg_sheet /
                                                (HBM_PEAK_GBS * 1e9), 5)},
            "stages_ms_per_step": {k: round(v / steps, 2) for k, v in totals.items()},
            "verified": checked, "mismatches": bad, "library": version, "valid": valid,
    }
    if bad:
        if d.rank == 0:
            print(json.dumps(line), flush=True)
        raise SystemExit("bench.py: %d C4 sheets differ from the oracle" % bad)
    return line


def main():
    args = parse()
    # Batches run on separate HIP streams so that one batch's latency-bound
    # sequential replays (one wave per sheet) overlap other batches' full-chip
    # kernels.  HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues
    # (default 4), read once at HIP init, i.e. in uphip_try_init below.
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, args.hw_queues)))
    d = Dist()
    L = load_library()
    version = L.uphip_version().decode()
    valid = diag_guard(version, os.environ, args.tuning)
    st = L.uphip_try_init()
    if st != 0:
        raise UnpaperHipError("no HIP device: " + L.uphip_init_status_string(st).decode())
    ndev = L.uphip_device_count()
    npages = args.pages or (16 if args.config == "c4" else 1000)
    devices, firsts, n_gpus = shard_plan(d.world, d.rank, d.local_rank, args.gpus, ndev, npages)
    if args.config == "c4":
        line = run_c4(args, L, d, devices, firsts, n_gpus, version, valid)
        if d.rank == 0:
            print(json.dumps(line), flush=True)
        return
    if args.config == "pdf":
        line = run_pdf(args, L, d, devices, firsts, n_gpus, version, valid)
        print(json.dumps(line))
        return
    if args.config in ("jpeg", "jp2"):
        line = run_jpeg(args, L, d, devices, firsts, n_gpus, version, valid, args.config)
        if d.rank == 0:
            print(json.dumps(line), flush=True)
        return

    bsz = max(1, min(args.batch or 64, npages))
    pitch = (W + 255) // 256 * 256
    stride = pitch * H
    bufs, shards = [], []
    for dev, first in zip(devices, firsts):
        L.uphip_set_device(dev)
        buf = DeviceBuffer(stride * npages)
        if L.uphip_synth_pages(buf.ptr, pitch, stride, W, H, first, npages) != 0:
            raise UnpaperHipError("synth_pages failed")
        bufs.append(buf)
        shards.append((buf.ptr, pitch, stride, npages))
    L.uphip_set_device(devices[0])
    opts = A.Options()
    L.uphip_options_init(C.byref(opts))     # the reference's defaults (lib/options.c)
    runner = Runner(opts, bsz, W, H, A.FMT_GRAY8, devices=devices, streams=max(1, args.streams),
                    timing=True)

    if args.warmup:
        failed, err = runner.run_device(shards, passes=args.warmup)
        if failed:
            raise UnpaperHipError("warm-up: %s" % err)
    stage_totals(runner, len(devices))          # drop the warm-up record
    d.barrier()
    t0 = time.perf_counter()
    failed, err = runner.run_device(shards, passes=args.steps)
    d.barrier()
    elapsed = d.max(time.perf_counter() - t0)
    if failed:
        raise UnpaperHipError("timed run: %d failed jobs: %s" % (failed, err))
    total_pages = d.sum(float(npages * args.steps * len(devices)))
    pages_per_s = total_pages / elapsed
    nchunks = (npages + bsz - 1) // bsz
    nlaunch = nchunks * args.steps * len(devices)

    checked = bad = 0
    if not args.no_verify:
        checked, bad = verify_resident(runner, devices, firsts, npages, bsz,
                                       load_hashes("bench_hashes.json", "pages"))
        checked, bad = int(d.sum(float(checked))), int(d.sum(float(bad)))

    totals = stage_totals(runner, len(devices))
    roofline = None
    if ROOFLINE_STAGE in totals:
        # In the timed region `streams` batches share the GPU, so one launch's
        # event span is stretched by the kernels of the other streams; the
        # kernel's own duration comes from probe launches right after it: the
        # same batch shape on one stream with the GPU otherwise idle.
        conc_ms = totals[ROOFLINE_STAGE] / max(nlaunch, 1)
        probe = probe_kernel(runner, shards[0], bsz, ROOFLINE_STAGE, args.probe)
        avg_ms = sum(probe) / len(probe) if probe else conc_ms
        units = bsz if probe else npages * args.steps * len(devices) / max(nlaunch, 1)
        alg = STAGE_PLANES[ROOFLINE_STAGE] * W * H * units
        achieved = alg / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        traffic, pipe_bytes = traffic_of(args.traffic, ROOFLINE_STAGE, units)
        roofline = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": ROOFLINE_KERNEL["c3"],
            "valu_issue_frac": valu_frac_of(args.valu, ROOFLINE_KERNEL["c3"], units, avg_ms),
            "alg_bytes_per_launch": int(alg), "avg_launch_ms": round(avg_ms, 3),
            "launch_ms_from": ("%d isolated probe launches of %d sheets" % (len(probe), bsz)
                               if probe else "timed region"),
            "concurrent_avg_launch_ms": round(conc_ms, 3),
            "pipeline_alg_bytes_per_page": ALG_BYTES_PER_PAGE,
            "pipeline_hbm_bytes_per_page": pipe_bytes,
            "pipeline_frac": round(pages_per_s / max(n_gpus, 1) * ALG_BYTES_PER_PAGE /
                                   (HBM_PEAK_GBS * 1e9), 5),
        }
    if args.stages and d.rank == 0:
        for k, v in sorted(totals.items(), key=lambda kv: -kv[1]):
            print("stage %-14s %9.1f ms total %8.3f ms/launch" % (k, v, v / max(nlaunch, 1)),
                  file=sys.stderr)
    runner.close()

    single = d.world == 1 and len(devices) == 1
    c4 = None
    if single and not args.no_c4:
        note("C3 done (%.0f pages/s); C4" % pages_per_s)
        # BASELINE configs[3] measured and verified in every default run: the
        # 16-sheet C4 workload, 1 warm-up + 3 timed passes
        c4 = run_c4(args, L, d, devices, [0], 1, version, valid, nsheets=16, steps=3, warmup=1,
                    batch=4)
        L.uphip_set_device(devices[0])
    threads = args.cpu_threads or host_threads_share()
    latency = hio = cpu = None
    host_pages = None
    if single and not (args.no_host_io and args.no_cpu and args.no_latency):
        host_pages = device_pages_to_host(L, bufs[0], pitch, stride, npages, W, H)
    if single and not args.no_latency:
        note("C2 latency")
        dev_ms, host_ms, stages = latency_c2(L, opts, host_pages[0], bufs[0].ptr, pitch, stride)
        latency = {"device_ms": dev_ms, "with_pcie_ms": host_ms,
                   "what": "one A4 GRAY8 page alone, idle GPU, median of 7 (C2)",
                   "stages_ms": stages}
    if single and not args.no_host_io:
        note("host-fed figures")
        hio = host_io(opts, devices[0], host_pages, npages, args, threads)
    if single and not args.no_cpu:
        note("CPU baseline")
        n = min(args.cpu_pages or 4 * threads, npages)
        v = cpu_baseline(host_pages, n, threads)
        n1 = min(3, npages)
        v1 = cpu_baseline(host_pages, n1, 1)
        # The reference's own --batch default is min(nproc, 64) worker
        # threads (lib/batch.c:72-83).  The box allots this job its CPU share
        # (OMP_NUM_THREADS), so the whole-host figure is the measured
        # one-thread rate times that thread count, with the measured scaling
        # of the share beside it.
        ref_threads = min(os.cpu_count() or 1, 64)
        cpu = {"value": round(v, 3), "unit": "pages/s", "cores": threads, "kind": "port",
               "host_cpus": os.cpu_count(),
               "sample": "%d synthetic A4 GRAY8 pages (the first of the GPU workload), default "
                         "options, oracle/oracle.c on %d host threads" % (n, threads),
               "one_thread": {"value": round(v1, 4), "cores": 1, "sample": "%d pages" % n1},
               "share_scaling": round(v / max(v1 * threads, 1e-9), 3),
               "whole_host": {"value": round(v1 * ref_threads, 2), "unit": "pages/s",
                              "cores": ref_threads, "kind": "port, extrapolated",
                              "how": "one-thread rate x min(nproc, 64) threads, the reference's "
                                     "batch default (lib/batch.c:72-83); not run at that width "
                                     "because the box allots this job %d CPUs" % threads}}
    for b in bufs:
        b.close()
    if d.rank == 0:
        out = {
            "metric": METRIC, "value": round(pages_per_s, 2), "unit": "pages/s",
            "n_gpus": n_gpus, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "mpixel_per_s": round(pages_per_s * W * H / 1e6, 1),
            "config": {"workload": "%d synthetic GRAY8 A4@300dpi pages (2480x3508) per GPU, "
                                   "default pipeline, inputs and outputs resident in HBM"
                                   % npages,
                       "pages_per_gpu": npages, "sheets_per_batch": bsz,
                       "streams": max(1, args.streams),
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "parallelism": ("one process per GPU (torchrun), pages sharded"
                                       if d.world > 1 else
                                       "one runner thread per device, pages sharded")
                       + ", no collective"},
            "roofline": roofline, "cpu_baseline": cpu, "latency_c2": latency, "host_io": hio,
            "c4": c4,
            "verified": checked, "mismatches": bad, "library": version, "valid": valid,
        }
        print(json.dumps(out), flush=True)
    d.close()
    if bad:
        raise SystemExit("bench.py: %d output pages differ from the oracle" % bad)


if __name__ == "__main__":
    main()
