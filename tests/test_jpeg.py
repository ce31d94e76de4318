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
