"""The GPU JPEG output branch (csrc/kernels_jpeg_enc.hip,
csrc/jpeg_enc.cpp, the runner's JPEG sink).

The reference encodes a finished device sheet with nvImageCodec
(src/core/sheet_stages.c:554-581 -> lib/encode_queue.c:860-990 ->
imageprocess/nvimgcodec.c:1007-1212), quality from --jpeg-quality (default 85).
nvImageCodec is not here, so its own bytes are unpinned; the encoder is pinned
to libjpeg-turbo, the IJG baseline encoder PIL links:

- CPU: oracle/jpeg_enc.c (the restatement, test infrastructure) equals PIL's
  output byte for byte (gray, 4:4:4, 4:2:2, 4:2:0; odd sizes; quality 1..100).
- GPU: uphip_jpeg_encode and the batch encode equal PIL byte for byte on
  the same pixels (so the quantised coefficients, Huffman codes, stuffing and
  headers all agree); a bit stream too large for the batch's buffers comes
  back for a single re-encode, with the same bytes.
- the reference's own acceptance criteria (tests/gpu_jpeg_pipeline_tests.py:
  199-330) through the runner: minimal pipeline SSIM >= 0.90 or diff <= 0.10
  and full pipeline SSIM >= 0.80 or diff <= 0.20 against the oracle's PNM,
  batch equals single, q60 files smaller than q95 -- plus the stronger check
  that the runner's files equal PIL's encode of the oracle's sheet.
"""
import ctypes as C
import io
import os

import numpy as np
import pytest
from PIL import Image

from unpaper_hip import ctypes_abi as A

ORACLE_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                         "_build", "liboracle.so")


def _oracle_lib():
    from oracle_py import Oracle
    L = Oracle().lib
    L.o_jpeg_encode.restype = C.c_int64
    L.o_jpeg_encode.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                C.c_void_p, C.c_int64]
    return L


def oracle_encode(a, quality, sampling):
    L = _oracle_lib()
    h, w = a.shape[:2]
    fmt = A.FMT_GRAY8 if a.ndim == 2 else A.FMT_RGB24
    a = np.ascontiguousarray(a)
    out = np.zeros(w * h * 8 + 65536, np.uint8)
    n = L.o_jpeg_encode(a.ctypes.data, a.strides[0], w, h, fmt, quality, sampling,
                        out.ctypes.data, out.size)
    assert n > 0
    return out[:n].tobytes()


def pil_encode(a, quality, sampling):
    b = io.BytesIO()
    kw = {} if a.ndim == 2 else {"subsampling": sampling}
    Image.fromarray(a).save(b, "JPEG", quality=quality, **kw)
    return b.getvalue()


def content(kind, w, h, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    if kind == "noise":
        return rng.integers(0, 256, (h, w, 3)).astype(np.uint8)
    if kind == "gradient":
        return np.stack([(x * 3 + y) % 256, (y * 5) % 256, (x * y) % 256], -1).astype(np.uint8)
    if kind == "text":  # white page, dark glyph-like runs, a light blotch
        a = np.full((h, w, 3), 255, np.uint8)
        for r in range(4, h - 8, 11):
            for c0 in range(3, w - 12, 17):
                if rng.random() < 0.7:
                    a[r:r + 6, c0:c0 + rng.integers(3, 12)] = rng.integers(0, 60)
        a[h // 3:h // 2, w // 4:w // 2] = (200, 190, 215)
        return a
    return np.full((h, w, 3), 77, np.uint8)  # uniform


SIZES = [(8, 8), (17, 9), (33, 47), (64, 64), (101, 77), (250, 131)]
MODES = ["L", 0, 1, 2]  # gray, 4:4:4, 4:2:2, 4:2:0


def _pick(a, mode):
    return np.ascontiguousarray(a[..., 0]) if mode == "L" else a


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("kind", ["noise", "gradient", "text", "uniform"])
def test_oracle_encoder_matches_pil(w, h, kind):
    """The restatement (oracle/jpeg_enc.c) is pinned to libjpeg-turbo."""
    base = content(kind, w, h, seed=w * h)
    for q in (1, 10, 50, 75, 85, 95, 100):
        for mode in MODES:
            a = _pick(base, mode)
            s = 0 if mode == "L" else mode
            assert oracle_encode(a, q, s) == pil_encode(a, q, s), (w, h, kind, q, mode)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------

def _device_image(a, pitch_pad=0):
    from unpaper_hip.pipeline import DeviceBuffer
    from unpaper_hip.device import load_library
    L = load_library()
    h = a.shape[0]
    row = a.shape[1] * (1 if a.ndim == 2 else 3)
    pitch = row + pitch_pad
    host = np.zeros((h, pitch), np.uint8)
    host[:, :row] = a.reshape(h, row)
    d = DeviceBuffer(pitch * h)
    assert L.uphip_memcpy_htod(d.ptr, host.ctypes.data, pitch * h) == 0
    return d, pitch


def device_encode(a, quality, sampling, pitch_pad=0):
    from unpaper_hip.pipeline import jpeg_encode
    d, pitch = _device_image(a, pitch_pad)
    fmt = A.FMT_GRAY8 if a.ndim == 2 else A.FMT_RGB24
    try:
        return jpeg_encode(d.ptr, pitch, a.shape[1], a.shape[0], fmt, quality, sampling)
    finally:
        d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("kind", ["noise", "gradient", "text", "uniform"])
def test_device_encode_matches_pil(hip, w, h, kind):
    base = content(kind, w, h, seed=w + h)
    for q in (1, 50, 85, 95, 100):
        for mode in MODES:
            a = _pick(base, mode)
            s = 0 if mode == "L" else mode
            for pad in (0, 256 - (a.shape[1] * (1 if a.ndim == 2 else 3)) % 256):
                got = device_encode(a, q, s, pad)
                assert got == pil_encode(a, q, s), (w, h, kind, q, mode, pad)


@pytest.mark.gpu
def test_device_encode_a4_pages(hip):
    """A synthetic A4 page (gray) and an RGB version of it (4:4:4 and 4:2:0),
    several tiles of 256 MCUs each, at the reference's default quality."""
    from unpaper_hip.pipeline import synth_page_host
    g = synth_page_host(2480, 3508, 3)
    assert device_encode(g, 85, 0) == pil_encode(g, 85, 0)
    rgb = np.stack([g, np.roll(g, 5, 1), np.maximum(g, 30)], 2)
    for s in (0, 2):
        assert device_encode(rgb, 85, s) == pil_encode(rgb, 85, s), s


@pytest.mark.gpu
def test_device_encode_default_quality_and_errors(hip):
    from unpaper_hip.device import load_library
    from unpaper_hip.pipeline import jpeg_encode
    a = content("text", 40, 30)[..., 0].copy()
    d, pitch = _device_image(a)
    try:
        assert jpeg_encode(d.ptr, pitch, 40, 30, A.FMT_GRAY8, 0, 0) == pil_encode(a, 85, 0)
        L = load_library()
        for args in ((pitch, 40, 30, A.FMT_GRAY8, 101, 0), (pitch, 40, 30, A.FMT_Y400A, 85, 0),
                     (pitch, 40, 30, A.FMT_RGB24, 85, 7), (10, 40, 30, A.FMT_GRAY8, 85, 0)):
            assert L.uphip_jpeg_encode(d.ptr, *args, None, 0) == -1, args
            assert L.uphip_last_error() is not None
            L.uphip_clear_error()
    finally:
        d.close()


def _batch_pages(w, h, n, seed):
    from unpaper_hip.pipeline import synth_page_host
    from unpaper_hip.hostimage import HostImage
    return [HostImage.from_array(synth_page_host(w, h, seed + i), A.FMT_GRAY8) for i in range(n)]


@pytest.mark.gpu
@pytest.mark.parametrize("quality,sampling", [(85, 0), (95, 2), (30, 1)])
def test_batch_encode_matches_pil(hip, oracle, quality, sampling):
    """The whole pipeline then the batch encode: every page's file equals
    PIL's encode of the batch's own output sheet (and the sheets equal the
    oracle's, as everywhere else)."""
    from unpaper_hip.pipeline import Batch
    w, h = 620, 877
    opts = oracle.default_options()
    pages = _batch_pages(w, h, 5, 40)
    b = Batch(opts, 5, w, h, A.FMT_GRAY8)
    try:
        for i, p in enumerate(pages):
            b.set_input(i, 0, p)
        b.run(5)
        b.encode_jpeg(quality, sampling)
        files = b.jpeg_files(5)
        for i in range(5):
            sheet = b.output(i)
            g = sheet.to_gray()
            assert files[i] == pil_encode(g, quality, sampling), i
    finally:
        b.close()


@pytest.mark.gpu
def test_batch_encode_rgb_two_output_pages(hip, oracle):
    """RGB24 working sheets (a coloured background), two output pages per
    sheet: each page encoded on its own, YCbCr 4:4:4 (nvImageCodec's
    default), equal to PIL's encode of that half of the batch's sheet."""
    from unpaper_hip.pipeline import Batch
    from unpaper_hip.hostimage import HostImage
    w, h = 300, 420
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.output_count = 2
    opts.sheet_background = A.Pixel(250, 240, 230)
    pages = [HostImage.from_array(np.stack([p.data[:, :w]] * 3, 2).copy(), A.FMT_RGB24)
             for p in _batch_pages(w, h, 3, 70)]
    b = Batch(opts, 3, w, h, A.FMT_RGB24)
    try:
        for i, p in enumerate(pages):
            b.set_input(i, 0, p)
        b.run(3)
        b.encode_jpeg(85, 0)
        files = b.jpeg_files(6)
        for s in range(3):
            rgb = b.output(s).to_rgb()
            half = rgb.shape[1] // 2
            for j in range(2):
                part = np.ascontiguousarray(rgb[:, j * half:(j + 1) * half])
                assert files[2 * s + j] == pil_encode(part, 85, 0), (s, j)
    finally:
        b.close()


@pytest.mark.gpu
def test_batch_encode_overflow_reencodes(hip, oracle):
    """Noise at quality 100 needs ~20 bits a pixel, more than the batch's
    per-page bit buffer (the page's bytes): the page comes back as -1 and the
    single-image path (uphip_batch_jpeg_page + uphip_jpeg_encode, exact
    buffers) gives PIL's bytes."""
    from unpaper_hip.pipeline import Batch, jpeg_encode
    from unpaper_hip.hostimage import HostImage
    w, h = 640, 480  # ~6 Mbit of codes against a 3 Mbit buffer (pixels + 64 KiB)
    opts = oracle.default_options()
    opts.disable = A.NO_PROCESSING
    rng = np.random.default_rng(5)
    noise = rng.integers(0, 256, (h, w)).astype(np.uint8)
    text = content("text", w, h)[..., 0].copy()
    b = Batch(opts, 2, w, h, A.FMT_GRAY8)
    try:
        b.set_input(0, 0, HostImage.from_array(noise, A.FMT_GRAY8))
        b.set_input(1, 0, HostImage.from_array(text, A.FMT_GRAY8))
        b.run(2)
        b.encode_jpeg(100, 0)
        files = b.jpeg_files(2)
        assert files[0] is None
        assert files[1] == pil_encode(text, 100, 0)
        src, pitch, pw, ph, fmt = b.jpeg_page(0)
        assert (pw, ph, fmt) == (w, h, A.FMT_GRAY8)
        assert jpeg_encode(src, pitch, pw, ph, fmt, 100, 0) == pil_encode(noise, 100, 0)
    finally:
        b.close()


# ---------------------------------------------------------------------------
# The reference's acceptance tests (gpu_jpeg_pipeline_tests.py:199-330)
# through the runner's JPEG sink
# ---------------------------------------------------------------------------

def _ssim(a1, a2):
    """gpu_jpeg_pipeline_tests.py:40-61 compute_ssim (global, grayscale)."""
    a1 = a1.astype(np.float64)
    a2 = a2.astype(np.float64)
    c1, c2 = (0.01 * 255) ** 2, (0.03 * 255) ** 2
    m1, m2 = a1.mean(), a2.mean()
    s1, s2 = ((a1 - m1) ** 2).mean(), ((a2 - m2) ** 2).mean()
    s12 = ((a1 - m1) * (a2 - m2)).mean()
    return ((2 * m1 * m2 + c1) * (2 * s12 + c2)) / ((m1 ** 2 + m2 ** 2 + c1) * (s1 + s2 + c2))


def _diff_ratio(a1, a2, threshold=30):
    """gpu_jpeg_pipeline_tests.py:64-85 compute_pixel_difference_ratio."""
    return float(np.mean(np.abs(a1.astype(np.int16) - a2.astype(np.int16)) > threshold))


def _run_jpeg_sink(opts, src_path, out_pattern, quality, sampling=0):
    from unpaper_hip.pipeline import Runner, image_read, sink_jpeg, source_pnm
    page = image_read(src_path)
    r = Runner(opts, 1, page.width, page.height, page.format, devices=(0,), streams=1,
               host_threads=2)
    try:
        failed, err = r.run_host(1, source_pnm([src_path]), sink_jpeg(out_pattern, 0, quality,
                                                                        sampling))
        assert failed == 0, err
    finally:
        r.close()
    return page


@pytest.mark.gpu
@pytest.mark.parametrize("minimal", [True, False])
def test_runner_jpeg_reference_criteria(hip, oracle, ref_path, tmp_path, minimal):
    """test_gpu_jpeg_minimal_matches_cpu / _full_matches_cpu: imgsrc001,
    --jpeg-quality 95; the CPU run's PNM (here the oracle's) vs the GPU run's
    JPEG.  Stronger: the JPEG equals PIL's encode (quality 95, one
    component) of the oracle's sheet."""
    opts = oracle.default_options()
    if minimal:
        opts.disable = A.NO_PROCESSING
    src = ref_path("imgsrc001.png")
    page = _run_jpeg_sink(opts, src, str(tmp_path / "gpu_%d.jpg"), 95)
    data = open(tmp_path / "gpu_0.jpg", "rb").read()
    sheet, fmt, _ = oracle.process_sheet(opts, [page])
    cpu = oracle.convert_for_save(sheet, fmt)  # the CPU run's .ppm / .pbm
    cpu_l = np.array(cpu.to_pil().convert("L"))
    gpu_l = np.array(Image.open(io.BytesIO(data)).convert("L"))
    assert gpu_l.shape == cpu_l.shape
    ssim, diff = _ssim(cpu_l, gpu_l), _diff_ratio(cpu_l, gpu_l)
    if minimal:
        assert ssim >= 0.90 or diff <= 0.10, (ssim, diff)
    else:
        assert ssim >= 0.80 or diff <= 0.20, (ssim, diff)
    assert data == pil_encode(sheet.to_gray(), 95, 0)


@pytest.mark.gpu
def test_runner_jpeg_batch_matches_single(hip, oracle, ref_path, tmp_path):
    """test_gpu_jpeg_batch_matches_single (quality 90): the runner's batch
    output equals the single-image encode of the same sheet, byte for byte
    (the reference allows SSIM 0.99)."""
    from unpaper_hip.pipeline import Batch, image_read
    opts = oracle.default_options()
    src = ref_path("imgsrc001.png")
    _run_jpeg_sink(opts, src, str(tmp_path / "batch_%04d.jpg"), 90)
    batch_file = open(tmp_path / "batch_0000.jpg", "rb").read()
    page = image_read(src)
    b = Batch(opts, 1, page.width, page.height, page.format)
    try:
        b.set_input(0, 0, page)
        b.run(1)
        b.wait()
        from unpaper_hip.pipeline import jpeg_encode
        single = jpeg_encode(*b.jpeg_page(0), 90, 0)
    finally:
        b.close()
    assert batch_file == single


@pytest.mark.gpu
def test_runner_jpeg_quality_affects_size(hip, oracle, ref_path, tmp_path):
    """test_gpu_jpeg_quality_affects_size: -n, q60 vs q95."""
    opts = oracle.default_options()
    opts.disable = A.NO_PROCESSING
    src = ref_path("imgsrc001.png")
    sizes = {}
    for q in (60, 95):
        _run_jpeg_sink(opts, src, str(tmp_path / ("q%d_%%d.jpg" % q)), q)
        sizes[q] = os.path.getsize(tmp_path / ("q%d_0.jpg" % q))
    assert sizes[60] < sizes[95], sizes


@pytest.mark.gpu
def test_runner_jpeg_sink_many_pages(hip, oracle, tmp_path):
    """A host-fed run of 70 synthetic pages over two batches of 64 and 6
    sheets into JPEG files: every file equals PIL's encode of the oracle's
    sheet."""
    from unpaper_hip.pipeline import Runner, sink_jpeg, source_memory
    w, h = 310, 440
    n = 70
    opts = oracle.default_options()
    pages = _batch_pages(w, h, n, 300)
    stack = np.stack([p.data[:, :w] for p in pages])
    r = Runner(opts, 64, w, h, A.FMT_GRAY8, devices=(0,), streams=2, host_threads=4)
    try:
        failed, err = r.run_host(n, source_memory(stack.ctypes.data, w, w * h, n, keep=stack),
                                 sink_jpeg(str(tmp_path / "p_%03d.jpg"), 0, 75, 0))
        assert failed == 0, err
    finally:
        r.close()
    for i in range(0, n, 7):
        sheet, _, _ = oracle.process_sheet(opts, [pages[i]])
        got = open(tmp_path / ("p_%03d.jpg" % i), "rb").read()
        assert got == pil_encode(sheet.to_gray(), 75, 0), i


def test_sink_jpeg_argument_checks():
    from unpaper_hip.device import load_library
    L = load_library()
    for args in ((b"x%d.jpg", 0, 101, 0), (b"x%d.jpg", 0, 85, 3), (b"x%s.jpg", 0, 85, 0)):
        assert not L.uphip_sink_jpeg(*args), args
        assert L.uphip_last_error() is not None
        L.uphip_clear_error()
    k = L.uphip_sink_jpeg(b"x%d.jpg", 0, 0, 2)
    assert k
    L.uphip_sink_destroy(k)
