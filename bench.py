#!/usr/bin/env python3
"""bench.py — pages/s of the per-sheet cleanup path on MI355X.

Workload (BASELINE.json configs[2], the metric's configuration): 1000
deterministic synthetic GRAY8 A4@300dpi pages (2480x3508)
per GPU, default unpaper options (the full sheet_process.c pipeline:
blackfilter, noisefilter, blurfilter, grayfilter, mask scan, deskew with
cubic rotation, mask centering, border scan), processed through the C-ABI
batch pipeline (uphip_batch_run_device) with a pool of batches on separate
HIP streams.  The pages are generated straight into HBM before the clock
starts; outputs stay in HBM (no PCIe inside the timed region).

One step = one pass of the pipeline over every page of the rank's shard.
N>1: one process per GPU (torch.distributed.run), pages sharded by rank with
no data-path collective; the gloo process group only provides the barrier
and the max-over-ranks of the elapsed time (weak scaling).

Extra fields: `roofline` for the dominant stage, timed live with the HIP
events the batch records on its own stream between stages; `cpu_baseline`
= the oracle's restatement of the reference CPU path, threaded over the host
cores, on a bounded sample of the same pages (rank 0, N=1 only).
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "unpaper-gpu_amd", "python"))

# The HIP library is loaded before torch so that one HIP runtime (/opt/rocm)
# serves the process; torch is only used for torch.distributed (gloo).
from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip.device import load_library, UnpaperHipError  # noqa: E402
from unpaper_hip.pipeline import Batch, DeviceBuffer  # noqa: E402

METRIC = "pages/sec + Mpixel/s, 1000-page GRAY8 A4@300dpi batch, 1/2/4/8 GPU"
W, H = 2480, 3508
HBM_PEAK_GBS = 8000.0                   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
ALG_BYTES_PER_PAGE = 10 * W * H         # SURVEY.md §8(d) fixed credit (86 998 400 B)

# Algorithmic HBM bytes per page of each timed stage (DESIGN.md "Kernels"):
# the bytes the stage must move at minimum, in units of one W*H GRAY8 plane.
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
ROOFLINE_KERNEL = "k_rotate_cubic_g8f"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pages", type=int, default=1000, help="pages per GPU")
    ap.add_argument("--batch", type=int, default=64, help="sheets per batch launch sequence")
    ap.add_argument("--streams", type=int, default=16, help="batches (HIP streams) in flight")
    ap.add_argument("--hw-queues", type=int, default=24,
                    help="GPU_MAX_HW_QUEUES for this process (HIP default 4, at most 32)")
    ap.add_argument("--cpu-pages", type=int, default=0,
                    help="CPU baseline sample (0 = 2 pages per host thread)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, host cores)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC HBM bytes per stage launch from a rocprofv3 --pmc pass")
    ap.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--probe", type=int, default=3,
                    help="isolated single-stream launches after the timed region that time "
                         "the roofline kernel (0 = use the concurrent timed-region spans)")
    ap.add_argument("--sweep", default="",
                    help="tuning only: comma list of BATCHxSTREAMS, each timed over one step "
                         "and printed to stderr before the main run")
    return ap.parse_args()


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def shard(rank, pages):
    """Pages of this rank: a contiguous block of the global job list."""
    return rank * pages, pages


def cpu_baseline(first_page, npages, threads):
    """The oracle (C restatement of the reference --device=cpu path), one page
    per thread at a time; ctypes releases the GIL inside the C call."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_py import Oracle
    from unpaper_hip.hostimage import HostImage
    from unpaper_hip.pipeline import synth_page_host
    oracle = Oracle()
    opts = oracle.default_options()
    pages = [HostImage.from_array(synth_page_host(W, H, first_page + i), A.FMT_GRAY8)
             for i in range(npages)]
    nxt = [0]
    lock = threading.Lock()

    def work():
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= npages:
                return
            oracle.process_sheet(opts, [pages[i]])

    ts = [threading.Thread(target=work) for _ in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return npages / (time.perf_counter() - t0)


def time_config(opts, pages, pitch, stride, npages, bsz, nstreams):
    """Seconds for one pass over the pages with a given batch/stream shape
    (after one warm-up pass)."""
    bs = [Batch(opts, bsz, W, H, A.FMT_GRAY8) for _ in range(nstreams)]
    chunks = [(s, min(bsz, npages - s)) for s in range(0, npages, bsz)]
    try:
        for rep in range(2):
            t0 = time.perf_counter()
            for i, (s, n) in enumerate(chunks):
                bs[i % nstreams].run_device(n, pages.ptr + s * stride, pitch, stride)
            for b in bs:
                b.wait()
            t = time.perf_counter() - t0
        return t
    finally:
        for b in bs:
            b.close()


def main():
    args = parse()
    # Batches run on separate HIP streams so that one batch's latency-bound
    # sequential replays (one wave per sheet) overlap other batches' full-chip
    # kernels.  HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues
    # (default 4), read once at HIP init, i.e. in uphip_try_init below.
    os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, min(32, args.hw_queues)))
    d = Dist()
    L = load_library()
    st = L.uphip_try_init()
    if st != 0:
        raise UnpaperHipError("no HIP device: " + L.uphip_init_status_string(st).decode())
    ndev = L.uphip_device_count()
    L.uphip_set_device(d.local_rank % max(ndev, 1))

    first, npages = shard(d.rank, args.pages)
    pitch = (W + 255) // 256 * 256
    stride = pitch * H
    pages = DeviceBuffer(stride * npages)
    if L.uphip_synth_pages(pages.ptr, pitch, stride, W, H, first, npages) != 0:
        raise UnpaperHipError("synth_pages failed")

    opts = A.Options()
    L.uphip_options_init(C.byref(opts))     # the reference's defaults (lib/options.c)
    for cfg in filter(None, args.sweep.split(",")):
        sb, ss = (int(v) for v in cfg.split("x"))
        t = time_config(opts, pages, pitch, stride, npages, sb, ss)
        print("sweep batch %d streams %d: %.1f pages/s" % (sb, ss, npages / t), file=sys.stderr,
              flush=True)
    bsz = max(1, min(args.batch, npages))
    batches = [Batch(opts, bsz, W, H, A.FMT_GRAY8, timing=True) for _ in range(max(1, args.streams))]
    chunks = [(s, min(bsz, npages - s)) for s in range(0, npages, bsz)]
    launches = [0]

    def step():
        for i, (s, n) in enumerate(chunks):
            batches[i % len(batches)].run_device(n, pages.ptr + s * stride, pitch, stride)
            launches[0] += 1

    def join():
        for b in batches:
            b.wait()

    for _ in range(args.warmup):
        step()
    join()
    for b in batches:
        b.stage_times()          # drop the warm-up record
    launches[0] = 0

    d.barrier()
    join()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    join()
    d.barrier()
    elapsed = d.max(time.perf_counter() - t0)

    # per-stage device time over the timed region (events on each batch's stream)
    totals = {}
    for b in batches:
        for name, ms in b.stage_times():
            totals[name] = totals.get(name, 0.0) + ms
    nlaunch = launches[0]
    total_pages = d.sum(float(npages * args.steps))
    pages_per_s = total_pages / elapsed
    mpix = pages_per_s * W * H / 1e6

    roofline = None
    if totals:
        # the dominant full-chip kernel: the bicubic rotation (its stage events
        # bracket exactly that launch); the one-wave/one-block sequential
        # replays are latency bound and overlap other streams' work
        dom = ROOFLINE_STAGE if ROOFLINE_STAGE in totals else max(totals, key=totals.get)
        # In the timed region `streams` batches share the GPU, so one launch's
        # event span is stretched by the kernels of the other streams.  The
        # kernel's own duration comes from probe launches right after the
        # timed region: the same batch shape on one stream with the GPU
        # otherwise idle (HIP events on that stream).
        conc_ms = totals[dom] / max(nlaunch, 1)
        n0 = chunks[0][1]
        probe = []
        for _ in range(args.probe):
            batches[0].run_device(n0, pages.ptr, pitch, stride)
            batches[0].wait()
            probe.append(sum(ms for name, ms in batches[0].stage_times() if name == dom))
        avg_ms = sum(probe) / len(probe) if probe else conc_ms
        units = n0 if probe else npages * args.steps / max(nlaunch, 1)
        alg = STAGE_PLANES.get(dom, 1.0) * W * H * units
        achieved = alg / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        traffic = None
        try:  # HBM bytes per page from the committed rocprofv3 --pmc passes
            with open(args.traffic) as f:
                per_page = json.load(f).get("bytes_per_page", {}).get(dom)
            if per_page:
                traffic = int(per_page * units)
        except (OSError, ValueError):
            pass
        roofline = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": ROOFLINE_KERNEL if dom == ROOFLINE_STAGE else dom,
            "alg_bytes_per_launch": int(alg), "avg_launch_ms": round(avg_ms, 3),
            "launch_ms_from": ("%d isolated probe launches of %d sheets" % (len(probe), n0)
                               if probe else "timed region"),
            "concurrent_avg_launch_ms": round(conc_ms, 3),
            "pipeline_frac": round(pages_per_s / max(d.world, 1) * ALG_BYTES_PER_PAGE /
                                   (HBM_PEAK_GBS * 1e9), 5),
        }
    if args.stages and d.rank == 0:
        for k, v in sorted(totals.items(), key=lambda kv: -kv[1]):
            print("stage %-14s %9.1f ms total %8.3f ms/launch" % (k, v, v / max(nlaunch, 1)),
                  file=sys.stderr)

    cpu = None
    if d.rank == 0 and d.world == 1 and not args.no_cpu:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        n = args.cpu_pages or 2 * threads
        v = cpu_baseline(first, n, threads)
        cpu = {"value": round(v, 3), "unit": "pages/s", "cores": threads, "kind": "port",
               "sample": "%d synthetic A4 GRAY8 pages (the first of the GPU workload), default "
                         "options, oracle/oracle.c on %d host threads" % (n, threads)}

    for b in batches:
        b.close()
    pages.close()
    if d.rank == 0:
        out = {
            "metric": METRIC, "value": round(pages_per_s, 2), "unit": "pages/s",
            "n_gpus": d.world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "mpixel_per_s": round(mpix, 1),
            "config": {"workload": "%d synthetic GRAY8 A4@300dpi pages (2480x3508) per GPU, "
                                   "default pipeline, batch_run_device" % args.pages,
                       "pages_per_gpu": args.pages, "sheets_per_batch": bsz,
                       "streams": len(batches),
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "parallelism": "pages sharded, no collective"},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()
