"""JPEG decode peer (csrc/jpeg.cpp + kernels_jpeg.hip).

Parity anchors:
- pixels: PIL's libjpeg-turbo (libjpeg's default islow IDCT, fancy
  upsampling, ycc_rgb_convert), byte for byte, for gray, 4:4:4, 4:2:2 and
  4:2:0 files, odd sizes, restart intervals, optimised Huffman tables,
  baseline and progressive (spectral selection, successive approximation).  The
  reference decodes with FFmpeg (file.c:29-128) or nvImageCodec
  (nvimgcodec.c:679-1007): parity with those decoders is unpinned.
- the reference's own acceptance test (tests/unpaper_tests.py:921-955):
  imgsrc001 saved by PIL as JPEG quality 95, filters and deskew off, output
  within 10 % (binarised compare_images) of the PNG run -- through the runner.

CPU tests: the host entropy decoder (uphip_jpeg_entropy_decode) plus a numpy
restatement of the pixel arithmetic (tests/jpeg_ref.py) against PIL.
GPU tests: the device path (uphip_jpeg_read / uphip_jpeg_decode, and runner
file sources) against PIL."""
import ctypes as C
import io
import os

import numpy as np
import pytest
from PIL import Image

import jpeg_ref
from unpaper_hip import ctypes_abi as A
from unpaper_hip.device import load_library


def _content(w, h, seed):
    rng = np.random.default_rng(seed)
    g = np.full((h, w), 255, np.uint8)
    g[h // 4:3 * h // 4, w // 5:4 * w // 5] = rng.integers(0, 256, (3 * h // 4 - h // 4,
                                                                  4 * w // 5 - w // 5))
    g = (g.astype(int) + np.add.outer(np.arange(h), np.arange(w)) % 50).clip(0, 255)
    return g.astype(np.uint8)


def make_jpeg(w, h, mode, seed=0, **kw):
    g = _content(w, h, seed)
    if mode == "L":
        im = Image.fromarray(g)
    else:
        im = Image.fromarray(np.stack([g, np.roll(g, 7, 1), 255 - g], 2))
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


def pil_decode(data):
    return np.asarray(Image.open(io.BytesIO(data)))


CASES = [
    ("L", 70, 50, dict(quality=90)),
    ("L", 333, 257, dict(quality=95)),
    ("L", 123, 77, dict(quality=75, optimize=True, restart_marker_rows=1)),
    ("RGB", 70, 50, dict(quality=90, subsampling=0)),
    ("RGB", 77, 41, dict(quality=90, subsampling=1)),
    ("RGB", 71, 53, dict(quality=90, subsampling=2)),
    ("RGB", 5, 9, dict(quality=90, subsampling=2)),      # downsampled width <= 2: box
    ("RGB", 300, 200, dict(quality=85, subsampling=2, restart_marker_blocks=3)),
    ("RGB", 257, 129, dict(quality=100, subsampling=0)),
    # progressive (SOF2): spectral selection + successive approximation
    # scans, end-of-band runs (libjpeg's jpeg_simple_progression script)
    ("L", 333, 257, dict(quality=95, progressive=True)),
    ("L", 70, 50, dict(quality=30, progressive=True, optimize=True)),
    ("RGB", 71, 53, dict(quality=90, subsampling=2, progressive=True)),
    ("RGB", 77, 41, dict(quality=90, subsampling=1, progressive=True)),
    ("RGB", 257, 129, dict(quality=100, subsampling=0, progressive=True)),
    ("RGB", 300, 200, dict(quality=85, subsampling=2, progressive=True,
                           restart_marker_blocks=3)),
]


@pytest.fixture(scope="module")
def lib():
    return load_library()


@pytest.mark.parametrize("mode,w,h,kw", CASES)
def test_host_decoder_with_reference_arithmetic_matches_pil(lib, mode, w, h, kw):
    data = make_jpeg(w, h, mode, seed=w, **kw)
    exp = pil_decode(data)
    got = jpeg_ref.decode(lib, data)
    assert got.shape == exp.shape
    assert np.array_equal(got, exp), np.count_nonzero(got != exp)


def _emulator():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "_build",
                        "libjdec_emul.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-s", "jdec_emul"],
                              cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    E = C.CDLL(path)
    E.jdec_emulate.restype = C.c_int64
    E.jdec_emulate.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64,
                               C.POINTER(C.c_int32)]
    return E


def emulate(data):
    E = _emulator()
    passes = C.c_int32()
    n = E.jdec_emulate(data, len(data), None, 0, C.byref(passes))
    if n < 0:
        from unpaper_hip.device import load_library
        load_library().uphip_clear_error()  # errors stick per thread until cleared
        return n, None, passes.value
    buf = np.zeros(n, np.uint8)
    assert E.jdec_emulate(data, len(data), buf.ctypes.data, n, C.byref(passes)) == n
    return n, buf, passes.value


SEQ_CASES = [c for c in CASES if not c[3].get("progressive")] + [
    ("L", 2480, 400, dict(quality=95)),     # many subsequences, no restarts
    ("RGB", 640, 480, dict(quality=75, subsampling=2, restart_marker_rows=1)),
    ("RGB", 333, 211, dict(quality=50, subsampling=1, optimize=True)),
    ("L", 1, 1, dict(quality=90)),
    ("L", 8, 8, dict(quality=100)),
]


@pytest.mark.parametrize("mode,w,h,kw", SEQ_CASES)
def test_device_huffman_decoder_emulated_matches_pil(lib, mode, w, h, kw):
    """The device entropy decoder's phases (kernels_jpeg_huff.hip) replayed on
    the CPU (tests/c/jdec_emul.cpp, same code) give PIL's pixels; the
    subsequence synchronisation converges within its passes."""
    data = make_jpeg(w, h, mode, seed=w + 1, **kw)
    n, buf, passes = emulate(data)
    assert n > 0, n
    got = jpeg_ref.decode_packed(buf)
    exp = pil_decode(data)
    assert np.array_equal(got, exp), np.count_nonzero(got != exp)
    hdr, _, (counts, groups, off) = jpeg_ref.planes(buf)
    per = hdr.scan[0].mcus_x * hdr.scan[0].blocks_per_mcu
    for g in range(hdr.ngroups):
        assert groups[g] == off[g * per]
    assert groups[-1] == counts.sum()
    assert passes >= 1, "no convergence within the sync passes (serial settle)"


def test_device_huffman_decoder_emulated_refusals(lib):
    """Progressive files stay with the host decoder (-2); corrupt data is
    reported, never silently decoded."""
    assert emulate(make_jpeg(64, 48, "RGB", quality=90, progressive=True))[0] == -2
    data = bytearray(make_jpeg(120, 90, "L", quality=90))
    sos = data.index(b"\xff\xda")
    for k in range(sos + 20, len(data) - 2, 7):
        data[k] ^= 0xA5
    n, _, _ = emulate(bytes(data))
    assert n < 0


def test_packed_layout_group_offsets(lib):
    """The per-MCU-row offsets the device prefix-sums from agree with the
    running count of coefficients (jpeg.h)."""
    data = make_jpeg(300, 200, "RGB", quality=85, subsampling=2)
    h, _, (counts, groups, off) = jpeg_ref.planes(jpeg_ref.entropy_decode(lib, data))
    assert h.nscans == 1 and h.scan[0].ncomp == 3 and h.scan[0].blocks_per_mcu == 6
    per = h.scan[0].mcus_x * h.scan[0].blocks_per_mcu
    assert len(groups) == h.ngroups + 1
    for g in range(h.ngroups):
        assert groups[g] == off[g * per]
    assert groups[-1] == counts.sum()


def test_probe(lib, tmp_path):
    for mode, fmt in (("L", A.FMT_GRAY8), ("RGB", A.FMT_RGB24)):
        p = tmp_path / ("x_%s.jpg" % mode)
        p.write_bytes(make_jpeg(91, 37, mode, quality=80))
        info = A.PnmInfo()
        assert lib.uphip_jpeg_probe(str(p).encode(), C.byref(info)) == 0
        assert (info.width, info.height, info.format) == (91, 37, fmt)
        info = A.PnmInfo()
        assert lib.uphip_image_probe(str(p).encode(), C.byref(info)) == 0
        assert info.format == fmt


@pytest.mark.parametrize("what,kw", [("truncated_progressive", dict(progressive=True)),
                                     ("truncated", None), ("garbage", None)])
def test_refused_files(lib, what, kw):
    if what == "truncated_progressive":
        data = make_jpeg(64, 64, "RGB", quality=90, **kw)
        data = data[:len(data) * 2 // 3]
    elif what == "truncated":
        data = make_jpeg(64, 64, "L", quality=90)[:40]
    else:
        data = b"\xff\xd8\xff" + bytes(np.random.default_rng(0).integers(0, 256, 500,
                                                                          dtype=np.uint8))
    assert lib.uphip_jpeg_entropy_decode(data, len(data), None, 0) == -1
    assert lib.uphip_last_error() is not None
    lib.uphip_clear_error()


# ---------------------------------------------------------------------------
# GPU: the device kernels
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("mode,w,h,kw", CASES)
def test_device_decode_matches_pil(hip, tmp_path, mode, w, h, kw):
    data = make_jpeg(w, h, mode, seed=w, **kw)
    exp = pil_decode(data)
    p = tmp_path / "in.jpg"
    p.write_bytes(data)
    L = hip.lib
    bpp = 1 if mode == "L" else 3
    ls = w * bpp + 5
    out = np.zeros((h, ls), np.uint8)
    assert L.uphip_jpeg_read(str(p).encode(), out.ctypes.data, ls, None) == 0, L.uphip_last_error()
    got = out[:, :w * bpp].reshape(exp.shape)
    assert np.array_equal(got, exp), np.count_nonzero(got != exp)


@pytest.mark.gpu
def test_device_decode_a4_gray_and_rgb(hip):
    """Page-sized inputs: an A4@300 gray page and a 4:2:0 colour page into
    device memory (uphip_jpeg_decode), against PIL."""
    from unpaper_hip.pipeline import DeviceBuffer, synth_page_host
    L = hip.lib
    g = synth_page_host(2480, 3508, 3)
    for mode, arr in (("L", g), ("RGB", np.stack([g, np.roll(g, 5, 0), g // 2 + 100], 2))):
        b = io.BytesIO()
        Image.fromarray(arr).save(b, "JPEG", quality=95)
        data = b.getvalue()
        exp = pil_decode(data)
        bpp = 1 if mode == "L" else 3
        pitch = (2480 * bpp + 255) // 256 * 256
        buf = DeviceBuffer(pitch * 3508)
        info = A.PnmInfo()
        assert L.uphip_jpeg_decode(data, len(data), buf.ptr, pitch, C.byref(info)) == 0, \
            L.uphip_last_error()
        host = np.empty((3508, pitch), np.uint8)
        assert L.uphip_memcpy_dtoh(host.ctypes.data, buf.ptr, host.nbytes) == 0
        buf.close()
        got = host[:, :2480 * bpp].reshape(exp.shape)
        assert np.array_equal(got, exp), (mode, np.count_nonzero(got != exp))


@pytest.mark.gpu
@pytest.mark.parametrize("mode,w,h,kw", SEQ_CASES)
def test_device_huffman_decode_matches_pil(hip, tmp_path, mode, w, h, kw):
    """One-scan sequential files take the device Huffman decoder
    (kernels_jpeg_huff.hip): pixels equal PIL's."""
    data = make_jpeg(w, h, mode, seed=w + 1, **kw)
    exp = pil_decode(data)
    L = hip.lib
    from unpaper_hip.pipeline import DeviceBuffer
    bpp = 1 if mode == "L" else 3
    pitch = (w * bpp + 255) // 256 * 256
    buf = DeviceBuffer(pitch * h)
    try:
        info = A.PnmInfo()
        assert L.uphip_jpeg_decode(data, len(data), buf.ptr, pitch, C.byref(info)) == 0, \
            L.uphip_last_error()
        host = np.empty((h, pitch), np.uint8)
        assert L.uphip_memcpy_dtoh(host.ctypes.data, buf.ptr, host.nbytes) == 0
    finally:
        buf.close()
    got = host[:, :w * bpp].reshape(exp.shape)
    assert np.array_equal(got, exp), np.count_nonzero(got != exp)


@pytest.mark.gpu
def test_device_huffman_decode_corrupt_data_fails_loudly(hip):
    """Bit errors in the entropy-coded data: the device decoder reports them
    (uphip_jpeg_decode returns -1 with a message), it never returns pixels
    silently -- unless the damaged stream still decodes (then it must equal
    PIL's decode of the same bytes)."""
    from unpaper_hip.pipeline import DeviceBuffer
    L = hip.lib
    data = bytearray(make_jpeg(120, 90, "L", quality=90))
    sos = data.index(b"\xff\xda")
    for k in range(sos + 20, len(data) - 2, 7):
        data[k] ^= 0xA5
    buf = DeviceBuffer(256 * 90)
    try:
        info = A.PnmInfo()
        rc = L.uphip_jpeg_decode(bytes(data), len(data), buf.ptr, 256, C.byref(info))
        assert rc == -1
        assert L.uphip_last_error() is not None
        L.uphip_clear_error()
    finally:
        buf.close()

