"""Host PNM codec (uphip_pnm_*), the file.c:29-259 peer: runs on the CPU.

Checks: write -> read round trips for the three direct formats
(saveImageDirect, file.c:133-176), byte-exact headers, PIL agreement on the
decoded pixels, the plain (ASCII) variants and comments, and loud failures on
malformed, truncated, 16-bit and mismatched files.
"""
import os

import numpy as np
import pytest

from unpaper_hip import ctypes_abi as AB
from unpaper_hip.device import UnpaperHipError, load_library
from unpaper_hip.hostimage import HostImage
from unpaper_hip.pipeline import pnm_read, pnm_write


def _img(fmt, w, h, seed):
    rng = np.random.default_rng(seed)
    if fmt == AB.FMT_GRAY8:
        return HostImage.from_array(rng.integers(0, 256, (h, w), dtype=np.uint8), fmt)
    if fmt == AB.FMT_RGB24:
        return HostImage.from_array(rng.integers(0, 256, (h, w, 3), dtype=np.uint8), fmt)
    return HostImage.from_array(rng.integers(0, 2, (h, w)).astype(bool), fmt)


@pytest.mark.parametrize("fmt,magic", [(AB.FMT_GRAY8, b"P5"), (AB.FMT_RGB24, b"P6"),
                                       (AB.FMT_MONOWHITE, b"P4")])
@pytest.mark.parametrize("w,h", [(1, 1), (13, 7), (64, 3), (301, 17)])
def test_roundtrip(tmp_path, fmt, magic, w, h):
    img = _img(fmt, w, h, w * 1000 + h)
    p = str(tmp_path / "x.pnm")
    pnm_write(p, img)
    raw = open(p, "rb").read()
    hdr = magic + b"\n%d %d\n" % (w, h) + (b"" if fmt == AB.FMT_MONOWHITE else b"255\n")
    assert raw.startswith(hdr)
    assert len(raw) == len(hdr) + img.payload().size
    back = pnm_read(p)
    assert (back.width, back.height, back.format) == (w, h, fmt)
    assert np.array_equal(back.payload(), img.payload())


def test_pil_agrees(tmp_path):
    from PIL import Image
    for fmt, mode in ((AB.FMT_GRAY8, "L"), (AB.FMT_RGB24, "RGB")):
        img = _img(fmt, 37, 11, 5)
        p = str(tmp_path / "y.pnm")
        pnm_write(p, img)
        with Image.open(p) as im:
            assert im.mode == mode
            assert np.array_equal(np.array(im).reshape(11, -1), img.payload())
    img = _img(AB.FMT_MONOWHITE, 37, 11, 6)
    p = str(tmp_path / "z.pbm")
    pnm_write(p, img)
    with Image.open(p) as im:
        assert np.array_equal(np.array(im.convert("L")), img.to_gray())


def test_plain_variants_and_comments(tmp_path):
    p = tmp_path / "a.pgm"
    p.write_bytes(b"P2\n# comment\n3 2 # trailing\n255\n0 1 2\n253 254\n255\n")
    g = pnm_read(str(p))
    assert g.format == AB.FMT_GRAY8
    assert g.payload().tolist() == [[0, 1, 2], [253, 254, 255]]
    p = tmp_path / "b.pbm"
    p.write_bytes(b"P1\n10 2\n1000000001\n01 0 1 0 1 0 1 0 0\n")
    m = pnm_read(str(p))
    assert m.format == AB.FMT_MONOWHITE
    assert m.payload().tolist() == [[0b10000000, 0b01000000], [0b01010101, 0b00000000]]
    p = tmp_path / "c.ppm"
    p.write_bytes(b"P3 2 1 255 1 2 3 4 5 6")
    c = pnm_read(str(p))
    assert c.format == AB.FMT_RGB24 and c.payload().tolist() == [[1, 2, 3, 4, 5, 6]]
    p = tmp_path / "d.pgm"   # comment between the header and a raw raster's separator
    p.write_bytes(b"P5 #x\n2 1\n255\n\x07\x08")
    assert pnm_read(str(p)).payload().tolist() == [[7, 8]]


@pytest.mark.parametrize("data,what", [
    (b"P5\n4 4\n255\n\x00\x01", "truncated"),
    (b"P5\n4 4\n65535\n" + b"\x00" * 32, "maxval"),
    (b"P7\n4 4\n255\n", "unsupported"),
    (b"XX", "not a PNM"),
    (b"P5\n-3 4\n255\n", "bad size"),
])
def test_malformed_fail_loudly(tmp_path, data, what):
    p = tmp_path / "bad.pnm"
    p.write_bytes(data)
    with pytest.raises(UnpaperHipError, match=what):
        pnm_read(str(p))


def test_geometry_mismatch_and_missing_file(tmp_path):
    import ctypes as C
    L = load_library()
    img = _img(AB.FMT_GRAY8, 8, 4, 1)
    p = str(tmp_path / "g.pgm")
    pnm_write(p, img)
    buf = np.zeros((4, 8), np.uint8)
    want = AB.PnmInfo(8, 5, AB.FMT_GRAY8)
    assert L.uphip_pnm_read(p.encode(), buf.ctypes.data, 8, C.byref(want)) != 0
    assert b"expected 8x5" in L.uphip_last_error()
    L.uphip_clear_error()
    with pytest.raises(UnpaperHipError, match="cannot open"):
        pnm_read(os.path.join(str(tmp_path), "missing.pgm"))
    with pytest.raises(UnpaperHipError, match="no direct PNM"):
        pnm_write(str(tmp_path / "q.pnm"), HostImage(4, 4, AB.FMT_Y400A))


def test_sink_pattern_integer_conversion_only():
    """the output pattern becomes a format string; reference-style
    "%04d" patterns are accepted (rewritten for the 64-bit page number), and
    anything but one integer conversion is refused at sink creation."""
    from unpaper_hip.device import load_library
    L = load_library()
    for good in (b"out%04d.pbm", b"p_%lld.pgm", b"x%u_%%.ppm", b"plain.pgm", b"o%-3ld.pgm"):
        h = L.uphip_sink_pnm(good, 0)
        assert h, good
        L.uphip_sink_destroy(h)
    for bad in (b"out%s.pgm", b"o%n.pgm", b"%d_%d.pgm", b"o%f.pgm", b"trail%"):
        L.uphip_clear_error()
        assert not L.uphip_sink_pnm(bad, 0), bad
        assert b"sink_pnm" in L.uphip_last_error()
    L.uphip_clear_error()
