"""The benchmarked configuration, the native runner and C4, on the GPU.

* bench configuration: bench.py itself (16 batches x 64 A4 sheets on their own
  streams, 24 HW queues, every batch re-run before the wait) in a subprocess
  (GPU_MAX_HW_QUEUES is read at HIP init); it hashes the resident outputs
  against tests/golden/bench_hashes.json (oracle, make_bench_hashes.py) and
  must report every checked page equal.
* runner (uphip_runner_*, the lib/batch_worker.c + decode/encode queue
  peer): host-fed runs through pinned staging against the oracle, PNM
  file-to-file, the reference's own PNG sources through the PNG decoder, the
  auto-sized batch layout, a failing source job isolated to itself, two and
  four runner threads on one device.
* C4 (BASELINE configs[3]): one RGB24 9920x7016 double-page sheet, layout
  double, bilinear deskew, border wipe, against the oracle's hash
  (tests/golden/c4_hashes.json).
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import assert_same
from unpaper_hip import ctypes_abi as A
from unpaper_hip.hostimage import HostImage
from unpaper_hip.pipeline import (Batch, DeviceBuffer, Runner, pnm_read, pnm_write, sink_memory,
                                  sink_pnm, source_callback, source_memory, source_pnm,
                                  synth_page_host)
from unpaper_hip.workloads import C4_H, C4_W, c4_options

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
SMALL = (620, 877)


def _bench(*extra, timeout=300):
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("UPHIP_DIAG"):
            del env[k]
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-host-io",
           "--no-latency", "--no-c4", "--probe", "0"] + list(extra)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_bench_configuration_matches_oracle():
    """The exact timed configuration: 1000 pages, 16 x 64-sheet batches, 2
    passes before the wait; the chunk each batch ran last is resident
    afterwards (chunks go to idle batches, so which varies) and every page of
    it is hashed against the oracle's (tests/golden/bench_hashes.json holds
    all 1000)."""
    out = _bench("--steps", "2", "--warmup", "1")
    assert out["config"]["sheets_per_batch"] == 64 and out["config"]["streams"] == 16
    assert out["config"]["hw_queues"] == 24
    assert out["valid"] is True
    assert out["verified"] >= 512 and out["mismatches"] == 0


def test_bench_four_streams_rerun_before_wait():
    """4 batches of 64 over 256 pages, 3 passes enqueued before one wait."""
    out = _bench("--pages", "256", "--streams", "4", "--steps", "3", "--warmup", "0")
    assert out["verified"] >= 64 and out["mismatches"] == 0


def _pages(n, first, w, h):
    return [HostImage.from_array(synth_page_host(w, h, first + i), A.FMT_GRAY8) for i in range(n)]


def _oracle_out(oracle, opts, page):
    sheet, fmt, _ = oracle.process_sheet(opts, [page])
    return oracle.convert_for_save(sheet, fmt)


def test_runner_host_fed_matches_oracle(hip, oracle):
    w, h = SMALL
    n = 11                                   # 3 chunks of 4, the last partial
    opts = oracle.default_options()
    pages = _pages(n, 40, w, h)
    host_in = np.stack([p.payload() for p in pages])
    r = Runner(opts, 4, w, h, A.FMT_GRAY8, devices=(0,), streams=2, host_threads=3)
    try:
        out = np.zeros((n, h, r.out_linesize), np.uint8)
        src = source_memory(host_in.ctypes.data, w, w * h, n, keep=host_in)
        snk = sink_memory(out.ctypes.data, r.out_linesize, r.out_linesize * h, n, keep=out)
        failed, err = r.run_host(n, src, snk)
        assert failed == 0, err
        st = r.stats()
        assert st.jobs_done == n and st.jobs_failed == 0 and st.jobs_per_device[0] == n
    finally:
        r.close()
    for i, p in enumerate(pages):
        exp = _oracle_out(oracle, opts, p)
        got = HostImage(w, h, exp.format, out[i])
        assert_same(got, exp, "runner job %d" % i)


@pytest.mark.parametrize("stride_kind", ["zero", "overlap"])
def test_runner_memory_source_overlapping_pages(hip, oracle, stride_kind):
    """a memory source whose pages overlap (page_stride 0 = one
    repeated page, or half a page) cannot be read in place by the batch; the
    runner takes the staged path and every job still gets its own page."""
    w, h = SMALL
    n = 3
    opts = oracle.default_options()
    stride = 0 if stride_kind == "zero" else w * (h // 2)
    rows = h + (n - 1) * (h // 2) if stride else h
    buf = np.full((rows, w), 255, np.uint8)
    buf[:h] = synth_page_host(w, h, 70)
    if stride:
        buf[h // 2:h // 2 + h] = np.minimum(buf[h // 2:h // 2 + h], synth_page_host(w, h, 71))
    flat = buf.reshape(-1)
    pages = [HostImage.from_array(flat[i * stride:i * stride + w * h].reshape(h, w).copy(),
                                  A.FMT_GRAY8) for i in range(n)]
    r = Runner(opts, 2, w, h, A.FMT_GRAY8, devices=(0,), streams=2, host_threads=2)
    try:
        out = np.zeros((n, h, r.out_linesize), np.uint8)
        src = source_memory(flat.ctypes.data, w, stride, n, keep=flat)
        snk = sink_memory(out.ctypes.data, r.out_linesize, r.out_linesize * h, n, keep=out)
        failed, err = r.run_host(n, src, snk)
        assert failed == 0, err
    finally:
        r.close()
    for i, p in enumerate(pages):
        exp = _oracle_out(oracle, opts, p)
        assert_same(HostImage(w, h, exp.format, out[i]), exp, "%s page %d" % (stride_kind, i))


def test_runner_numa_placement(hip):
    import ctypes
    """VERDICT r03 item 7: each device's thread and load/store pool are bound
    to the CPUs of the GPU's NUMA node (sysfs via the PCI bus id), and the
    pool threads split the host threads between devices."""
    w, h = SMALL
    opts = A.Options()
    hip.lib.uphip_options_init(ctypes.byref(opts))
    r = Runner(opts, 2, w, h, A.FMT_GRAY8, devices=(0, 0), streams=1, host_threads=5)
    try:
        pl = [r.placement(i) for i in range(2)]
    finally:
        r.close()
    assert sorted(p[2] for p in pl) == [2, 3]
    bus = ctypes_bus_id(hip.lib, 0)
    node_file = "/sys/bus/pci/devices/%s/numa_node" % bus.lower()
    node = int(open(node_file).read()) if os.path.exists(node_file) else -1
    for n, ncpu, _ in pl:
        if node >= 0:
            assert n == node and ncpu > 0, (pl, node)
        else:
            assert n == -1 and ncpu == 0, (pl, node)


def ctypes_bus_id(lib, dev):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    assert hip.hipDeviceGetPCIBusId(buf, 63, dev) == 0
    return buf.value.decode()


def test_runner_pnm_files(hip, oracle, tmp_path):
    """Decode queue -> device -> encode queue: PGM in, PGM out."""
    w, h = SMALL
    n = 5
    opts = oracle.default_options()
    pages = _pages(n, 60, w, h)
    paths = []
    for i, p in enumerate(pages):
        q = str(tmp_path / ("in_%d.pgm" % i))
        pnm_write(q, p)
        paths.append(q)
    r = Runner(opts, 2, w, h, A.FMT_GRAY8, devices=(0,), streams=2, host_threads=2)
    try:
        failed, err = r.run_host(n, source_pnm(paths), sink_pnm(str(tmp_path / "out_%03lld.pgm")))
        assert failed == 0, err
    finally:
        r.close()
    for i, p in enumerate(pages):
        got = pnm_read(str(tmp_path / ("out_%03d.pgm" % i)))
        assert_same(got, _oracle_out(oracle, opts, p), "pnm job %d" % i)


def test_runner_auto_layout(hip, oracle):
    """sheets=0, streams=0: the runner sizes its batches (the reference's VRAM
    tiers, image_pipeline.c:237-285): 2 GiB of input + two planes per batch
    at most 64 sheets, batches until half the free memory, at most 16."""
    w, h = SMALL
    opts = oracle.default_options()
    r = Runner(opts, 0, w, h, A.FMT_GRAY8, devices=(0,), streams=0, host_threads=2)
    try:
        per_sheet = ((w + 255) & ~255) * h + 2 * w * h
        assert r.geometry.capacity == min(64, (2 << 30) // per_sheet)
        assert 1 <= r.streams <= 16 and r.batch_bytes >= per_sheet * r.geometry.capacity
        n = 5
        pages = _pages(n, 70, w, h)
        host_in = np.stack([p.payload() for p in pages])
        out = np.zeros((n, h, r.out_linesize), np.uint8)
        failed, err = r.run_host(n, source_memory(host_in.ctypes.data, w, w * h, n, keep=host_in),
                                 sink_memory(out.ctypes.data, r.out_linesize, r.out_linesize * h,
                                             n, keep=out))
        assert failed == 0, err
    finally:
        r.close()
    for i, p in enumerate(pages):
        exp = _oracle_out(oracle, opts, p)
        assert_same(HostImage(w, h, exp.format, out[i]), exp, "auto layout job %d" % i)
    # a C4-sized RGB24 sheet pair gets few sheets per batch
    big = Runner(c4_options(oracle.default_options()), 0, C4_W, C4_H, A.FMT_RGB24, devices=(0,),
                 streams=2)
    try:
        per_sheet = ((C4_W * 3 + 255) & ~255) * C4_H + 2 * 3 * C4_W * C4_H
        assert big.geometry.capacity == max(1, min(64, (2 << 30) // per_sheet))
        assert big.streams == 2
    finally:
        big.close()


@pytest.mark.parametrize("names,fmt,out_ext", [
    (("imgsrc002.png", "imgsrc005.png"), A.FMT_MONOBLACK, "pbm"),
    (("imgsrc004.png",), A.FMT_GRAY8, "pgm"),
    (("imgsrc003.png",), A.FMT_RGB24, "ppm")])
def test_runner_png_reference_sources(hip, oracle, ref_path, tmp_path, names, fmt, out_ext):
    """The reference's own PNG test sources (1-bit -> MONOBLACK, gray, RGB)
    decoded by the native PNG codec straight into staging, processed with
    default options and written as PNM, against the oracle on the same pages
    loaded through PIL."""
    opts = oracle.default_options()
    pages = [HostImage.load(ref_path(n)) for n in names]
    w, h = pages[0].width, pages[0].height
    assert all(p.format == fmt for p in pages)
    r = Runner(opts, 2, w, h, fmt, devices=(0,), streams=1, host_threads=2)
    try:
        failed, err = r.run_host(len(names), source_pnm([ref_path(n) for n in names]),
                                 sink_pnm(str(tmp_path / ("out_%02d." + out_ext))))
        assert failed == 0, err
    finally:
        r.close()
    for i, p in enumerate(pages):
        got = pnm_read(str(tmp_path / ("out_%02d.%s" % (i, out_ext))))
        assert_same(got, _oracle_out(oracle, opts, p), "png job %s" % names[i])


def _no_filters(opts):
    """The reference JPEG test's option set (unpaper_tests.py:941-948)."""
    opts.disable |= (A.NO_BLACKFILTER | A.NO_NOISEFILTER | A.NO_BLURFILTER | A.NO_GRAYFILTER |
                     A.NO_DESKEW)
    return opts


def test_runner_jpeg_reference_acceptance(hip, oracle, ref_path, tmp_path):
    """The reference's own JPEG acceptance test (tests/unpaper_tests.py:921-955)
    through the runner's JPEG path (host entropy decode into pinned memory,
    device IDCT into the batch's input slot): imgsrc001 saved by PIL as JPEG
    quality 95 (a grayscale JPEG: PIL writes mode "1" as L), filters and
    deskew off, output within 10 % (binarised compare_images) of the PNG run.
    Stronger: the JPEG run equals the oracle on PIL's decode of the same file
    byte for byte (device pixels == libjpeg's, pipeline == oracle)."""
    from PIL import Image
    from unpaper_hip.hostimage import binarized_diff_ratio
    opts = _no_filters(oracle.default_options())
    src = ref_path("imgsrc001.png")
    jpg = tmp_path / "source.jpg"
    Image.open(src).save(jpg, "JPEG", quality=95)
    pil = np.asarray(Image.open(jpg))
    assert pil.ndim == 2
    h, w = pil.shape
    r = Runner(opts, 1, w, h, A.FMT_GRAY8, devices=(0,), streams=1, host_threads=2)
    try:
        failed, err = r.run_host(1, source_pnm([str(jpg)]), sink_pnm(str(tmp_path / "jpg_%d.pgm")))
        assert failed == 0, err
    finally:
        r.close()
    got = pnm_read(str(tmp_path / "jpg_0.pgm"))
    exp = _oracle_out(oracle, opts, HostImage.from_array(pil.copy(), A.FMT_GRAY8))
    assert_same(got, exp, "jpeg page vs oracle on PIL's decode")
    png_page = HostImage.load(src)
    png_out = _oracle_out(oracle, opts, png_page)
    ratio = binarized_diff_ratio(np.array(got.to_pil().convert("L")),
                                 np.array(png_out.to_pil().convert("L")))
    assert ratio < 0.10, ratio


def test_runner_jpeg_colour_and_mixed_sources(hip, oracle, tmp_path):
    """A runner chunk mixing JPEG (4:2:0 and 4:4:4) and PNM pages of one
    RGB24 geometry: every page through its own decoder, JPEG pages decoded on
    the slot's stream into their input slots; outputs against the oracle on
    PIL's decode."""
    from PIL import Image
    w, h = SMALL
    opts = oracle.default_options()
    paths, pages = [], []
    for i in range(5):
        g = synth_page_host(w, h, 90 + i)
        rgb = np.stack([g, np.roll(g, 3, 1), np.maximum(g, 40)], 2)
        if i == 2:
            q = str(tmp_path / ("p%d.ppm" % i))
            pnm_write(q, HostImage.from_array(rgb, A.FMT_RGB24))
            px = rgb
        else:
            q = str(tmp_path / ("p%d.jpg" % i))
            Image.fromarray(rgb).save(q, "JPEG", quality=92, subsampling=2 if i % 2 else 0)
            px = np.asarray(Image.open(q))
        paths.append(q)
        pages.append(HostImage.from_array(px.copy(), A.FMT_RGB24))
    r = Runner(opts, 3, w, h, A.FMT_RGB24, devices=(0,), streams=2, host_threads=3)
    try:
        failed, err = r.run_host(len(paths), source_pnm(paths), sink_pnm(str(tmp_path / "o%02d.ppm")))
        assert failed == 0, err
    finally:
        r.close()
    for i, p in enumerate(pages):
        assert_same(pnm_read(str(tmp_path / ("o%02d.ppm" % i))), _oracle_out(oracle, opts, p),
                    "page %d (%s)" % (i, paths[i]))


def test_runner_two_outputs_pbm(hip, oracle, tmp_path):
    """--layout double --output-pages 2 with MONOWHITE output: the encode
    queue splits every sheet into two PBM pages (sheet_stages.c:606-624)."""
    w, h = SMALL
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.output_count = 2
    opts.output_pixel_format = A.FMT_MONOWHITE
    pages = _pages(2, 80, w + 3, h)        # odd half width: unaligned PBM split
    host_in = np.stack([p.payload() for p in pages])
    r = Runner(opts, 2, w + 3, h, A.FMT_GRAY8, devices=(0,), streams=1, host_threads=2)
    try:
        src = source_memory(host_in.ctypes.data, w + 3, (w + 3) * h, 2, keep=host_in)
        failed, err = r.run_host(2, src, sink_pnm(str(tmp_path / "p_%lld.pbm")))
        assert failed == 0, err
    finally:
        r.close()
    for i, p in enumerate(pages):
        sheet = _oracle_out(oracle, opts, p)
        half = sheet.width // 2
        g = sheet.to_gray()
        for j in range(2):
            got = pnm_read(str(tmp_path / ("p_%d.pbm" % (2 * i + j))))
            assert (got.width, got.height, got.format) == (half, h, A.FMT_MONOWHITE)
            assert np.array_equal(got.to_gray(), g[:, j * half:(j + 1) * half]), (i, j)


def test_runner_failed_job_is_isolated(hip, oracle):
    """A job whose page cannot be loaded fails alone (batch_worker.c:214-231:
    the job is marked failed, the others complete)."""
    w, h = SMALL
    n = 6
    opts = oracle.default_options()
    pages = _pages(n, 90, w, h)
    import ctypes as C

    def load(job, page, dst, linesize):
        if job == 4:
            return 1
        a = pages[job].payload()
        for y in range(h):
            C.memmove(dst + y * linesize, a[y].ctypes.data, w)
        return 0

    r = Runner(opts, 3, w, h, A.FMT_GRAY8, devices=(0,), streams=2, host_threads=2)
    try:
        out = np.zeros((n, h, r.out_linesize), np.uint8)
        snk = sink_memory(out.ctypes.data, r.out_linesize, r.out_linesize * h, n, keep=out)
        failed, err = r.run_host(n, source_callback(load), snk)
        assert failed == 1 and "could not be loaded" in err
        assert r.stats().jobs_done == n - 1
    finally:
        r.close()
    for i in (0, 3, 5):
        exp = _oracle_out(oracle, opts, pages[i])
        assert_same(HostImage(w, h, exp.format, out[i]), exp, "job %d" % i)
    assert not out[4].any()


def test_runner_two_threads_one_device(hip, oracle):
    """Two runner device threads bound to the same GPU (the multi-device
    fan-out path): disjoint device-resident shards, per-thread batches."""
    w, h = SMALL
    n = 6
    opts = oracle.default_options()
    pitch = (w + 255) // 256 * 256
    bufs = []
    for first in (100, 200):
        b = DeviceBuffer(pitch * h * n)
        assert b.lib.uphip_synth_pages(b.ptr, pitch, pitch * h, w, h, first, n) == 0
        bufs.append(b)
    r = Runner(opts, 4, w, h, A.FMT_GRAY8, devices=(0, 0), streams=2)
    try:
        failed, err = r.run_device([(b.ptr, pitch, pitch * h, n) for b in bufs], passes=2)
        assert failed == 0, err
        st = r.stats()
        assert st.jobs_per_device[0] == 2 * n and st.jobs_per_device[1] == 2 * n
        # each batch holds the chunk it ran last (chunks go to idle batches):
        # between them the two batches of a thread hold chunk 0 (sheets 0..3)
        # and chunk 1 (4..5)
        for i, first in enumerate((100, 200)):
            held = sorted(r.slot_chunk(i, k) + (k,) for k in range(2))
            assert [h[:2] for h in held] == [(0, 4), (4, 2)], held
            for c0, cnt, k in held:
                b = r.batch(i, k)
                for s in range(cnt):
                    exp = _oracle_out(oracle, opts, _pages(1, first + c0 + s, w, h)[0])
                    assert_same(b.output(s), exp, "thread %d sheet %d" % (i, c0 + s))
    finally:
        r.close()
        for b in bufs:
            b.close()


def test_runner_four_device_threads_host_fed(hip, tmp_path):
    """Multi-GPU readiness on one GPU: run_host with four device
    threads (devices=(0,0,0,0)) pulling 2-sheet chunks from the one shared job
    counter (the BatchQueue peer, batch_worker.c:174-263), PGM files in and
    out, one job whose file is missing.  The failed job is isolated, every
    other output file is named by its job index and equals the oracle's hash
    of that A4 page, and the per-device counters add up."""
    hashes = json.load(open(os.path.join(GOLDEN, "bench_hashes.json")))["pages"]
    from unpaper_hip.workloads import A4_H, A4_W
    import ctypes as C
    L = hip.lib
    opts = A.Options()
    L.uphip_options_init(C.byref(opts))
    n, bad = 22, 13
    paths = []
    for p in range(n):
        q = str(tmp_path / ("in_%02d.pgm" % p))
        if p != bad:
            pnm_write(q, HostImage.from_array(synth_page_host(A4_W, A4_H, p), A.FMT_GRAY8))
        paths.append(q)
    r = Runner(opts, 2, A4_W, A4_H, A.FMT_GRAY8, devices=(0, 0, 0, 0), streams=2, host_threads=8)
    try:
        failed, err = r.run_host(n, source_pnm(paths), sink_pnm(str(tmp_path / "out_%03d.pgm")))
        st = r.stats()
    finally:
        r.close()
    assert failed == 1 and "could not be loaded" in err
    assert st.jobs_done == n - 1 and st.jobs_failed == 1
    per = [st.jobs_per_device[i] for i in range(4)]
    assert sum(per) == n - 1 and sum(1 for v in per if v) >= 2, per
    assert not os.path.exists(str(tmp_path / ("out_%03d.pgm" % bad)))
    for p in range(n):
        if p == bad:
            continue
        got = pnm_read(str(tmp_path / ("out_%03d.pgm" % p)))
        assert (got.width, got.height, got.format) == (A4_W, A4_H, A.FMT_GRAY8)
        assert hashlib.sha256(got.payload().tobytes()).hexdigest() == hashes[str(p)], p


def test_output_right_after_run_monowhite(hip, oracle):
    """output() straight after run(), no wait, with a converted
    (MONOWHITE) output: the read must be ordered after the output kernel."""
    w, h = SMALL
    opts = oracle.default_options()
    opts.output_pixel_format = A.FMT_MONOWHITE
    pages = _pages(3, 7, w, h)
    b = Batch(opts, 3, w, h, A.FMT_GRAY8)
    try:
        for s, p in enumerate(pages):
            b.set_input(s, 0, p)
        b.run(3)
        outs = [b.output(s) for s in range(3)]
    finally:
        b.close()
    for s, p in enumerate(pages):
        assert_same(outs[s], _oracle_out(oracle, opts, p), "sheet %d" % s)


def _c4_hashes():
    with open(os.path.join(GOLDEN, "c4_hashes.json")) as f:
        return json.load(f)["sheets"]


def test_c4_double_page_rgb_matches_oracle(hip):
    """BASELINE configs[3]: RGB24 600dpi double-page scans through the full
    pipeline (layout double, bilinear deskew, border wipe): every sheet of the
    bench's C4 workload that has an oracle hash, in 4-sheet batches as the
    bench runs them.  The odd sheets carry the dark band, and some of those
    grow blackfilter fills of thousands of frames (the replay's driver/helper
    path, its LDS and HBM stack)."""
    import ctypes as C
    L = hip.lib
    opts = A.Options()
    L.uphip_options_init(C.byref(opts))
    c4_options(opts)
    want = _c4_hashes()
    nsheets = len(want)
    pitch = (3 * C4_W + 255) // 256 * 256
    buf = DeviceBuffer(pitch * C4_H * nsheets)
    assert L.uphip_synth_sheets_rgb(buf.ptr, pitch, pitch * C4_H, C4_W, C4_H, 0, nsheets) == 0
    bsz = min(4, nsheets)
    b = Batch(opts, bsz, C4_W, C4_H, A.FMT_RGB24)
    try:
        for first in range(0, nsheets, bsz):
            n = min(bsz, nsheets - first)
            b.run_device(n, buf.ptr + first * pitch * C4_H, pitch, pitch * C4_H)
            b.wait()
            for s in range(n):
                out = b.output(s)
                assert (out.width, out.height, out.format) == (C4_W, C4_H, A.FMT_RGB24)
                got = hashlib.sha256(out.payload().tobytes()).hexdigest()
                assert got == want[str(first + s)], first + s
                rep = b.report(s)
                assert rep.mask_count == 2            # one mask per page of the double layout
    finally:
        b.close()
        buf.close()


def test_c4_synth_device_matches_host(hip):
    """The C4 generator is identical on host and device (a band of rows)."""
    from unpaper_hip.pipeline import synth_sheet_rgb_host
    w, h = 998, 64
    pitch = (3 * w + 255) // 256 * 256
    buf = DeviceBuffer(pitch * h)
    L = buf.lib
    assert L.uphip_synth_sheets_rgb(buf.ptr, pitch, pitch * h, w, h, 3, 1) == 0
    host = np.empty((h, pitch), np.uint8)
    assert L.uphip_memcpy_dtoh(host.ctypes.data, buf.ptr, host.nbytes) == 0
    assert np.array_equal(host[:, :3 * w], synth_sheet_rgb_host(w, h, 3).reshape(h, 3 * w))
    buf.close()
