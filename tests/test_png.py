"""Host PNG decoder (uphip_png_*, uphip_image_*), the PNG half of loadImage
(file.c:29-131): runs on the CPU.

Checks:
- the reference's own PNG sources and goldens (tests/imgsrc*.png, re-encoded
  under tests/golden/reference) decode to the same pixels and format as
  HostImage.load (PIL), the format mapping FFmpeg gives loadImage;
- files written by an independent encoder below (every colour type and bit
  depth the mapping names, all five filter types, Adam7) decode to the
  expected rows: 1-bit gray -> MONOBLACK, 2/4-bit gray scaled by 0x55/0x11,
  palette -> RGB24 with out-of-range indices black, gray + tRNS -> Y400A;
- loud failures for 16-bit, RGBA, RGB + tRNS, truncated and corrupt data,
  geometry mismatch; uphip_image_* dispatches on the signature.
The 2/4-bit scaling and the tRNS cases follow FFmpeg's pngdec and have no
fixture in the reference: parity unpinned for those two rows.
"""
import struct
import zlib

import numpy as np
import pytest

from unpaper_hip import ctypes_abi as AB
from unpaper_hip.device import UnpaperHipError, load_library
from unpaper_hip.hostimage import HostImage
from unpaper_hip.pipeline import image_read, pnm_write

import ctypes as C

ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
         (0, 1, 1, 2)]


def _chunk(t, data):
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data))


def _filter_row(raw, prev, bpp, ftype):
    out = bytearray(len(raw))
    for i in range(len(raw)):
        a = raw[i - bpp] if i >= bpp else 0
        b = prev[i]
        c = prev[i - bpp] if i >= bpp else 0
        if ftype == 0:
            p = 0
        elif ftype == 1:
            p = a
        elif ftype == 2:
            p = b
        elif ftype == 3:
            p = (a + b) // 2
        else:
            pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
            p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (raw[i] - p) & 0xFF
    return bytes([ftype]) + bytes(out)


def _pack_row(samples, depth):
    """samples: 1-D int array of one row's samples -> packed bytes."""
    if depth == 8:
        return bytes(np.asarray(samples, dtype=np.uint8))
    if depth == 16:
        return np.asarray(samples, dtype=">u2").tobytes()
    per = 8 // depth
    n = len(samples)
    out = bytearray((n * depth + 7) // 8)
    for i, v in enumerate(samples):
        out[i // per] |= int(v) << (8 - depth * (i % per + 1))
    return bytes(out)


def write_png(path, samples, depth, ctype, interlace=False, plte=None, trns=None, seed=0):
    """samples: (H, W, channels) int array of raw sample values."""
    h, w, ch = samples.shape
    bpp = max(1, ch * depth // 8)
    rng = np.random.default_rng(seed)

    def encode(img):
        rows = []
        prev = bytes(((img.shape[1] * ch * depth) + 7) // 8)
        for y in range(img.shape[0]):
            raw = _pack_row(img[y].reshape(-1), depth)
            rows.append(_filter_row(raw, prev, bpp, int(rng.integers(0, 5))))
            prev = raw
        return b"".join(rows)

    if interlace:
        data = b""
        for x0, y0, dx, dy in ADAM7:
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                data += encode(sub)
    else:
        data = encode(samples)
    out = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0,
                                                          1 if interlace else 0))
    if plte is not None:
        out += _chunk(b"PLTE", bytes(np.asarray(plte, dtype=np.uint8).reshape(-1)))
    if trns is not None:
        out += _chunk(b"tRNS", trns)
    z = zlib.compress(data, 6)
    # split the stream over several IDAT chunks
    cuts = sorted(set([0, len(z)] + [int(c) for c in rng.integers(0, len(z), 3)]))
    for a, b in zip(cuts, cuts[1:]):
        out += _chunk(b"IDAT", z[a:b])
    out += _chunk(b"IEND", b"")
    open(path, "wb").write(out)


def _decoded(p):
    img = image_read(str(p))
    n = {AB.FMT_GRAY8: 1, AB.FMT_Y400A: 2, AB.FMT_RGB24: 3}.get(img.format)
    return img, n


@pytest.mark.parametrize("name", ["imgsrc001.png", "imgsrc002.png", "imgsrc003.png",
                                  "imgsrc004.png", "imgsrc005.png", "imgsrc006.png",
                                  "imgsrcE001.png", "goldenC1_ppm.png", "goldenF_pbm.png"])
def test_reference_fixtures_match_pil(ref_path, name):
    want = HostImage.load(ref_path(name))
    got = image_read(ref_path(name))
    assert (got.width, got.height, got.format) == (want.width, want.height, want.format)
    assert np.array_equal(got.payload(), want.payload())


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("w,h", [(1, 1), (5, 3), (37, 19), (64, 9)])
def test_gray8_rgb24_y400a(tmp_path, interlace, w, h):
    rng = np.random.default_rng(w * 100 + h)
    for ctype, ch, fmt in ((0, 1, AB.FMT_GRAY8), (2, 3, AB.FMT_RGB24), (4, 2, AB.FMT_Y400A)):
        s = rng.integers(0, 256, (h, w, ch))
        p = tmp_path / ("c%d.png" % ctype)
        write_png(p, s, 8, ctype, interlace, seed=ctype)
        img, n = _decoded(p)
        assert (img.width, img.height, img.format) == (w, h, fmt)
        assert np.array_equal(img.payload(), s.reshape(h, w * n).astype(np.uint8))


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("w,h", [(1, 1), (9, 4), (33, 17), (64, 8)])
def test_monoblack(tmp_path, interlace, w, h):
    s = np.random.default_rng(w + h).integers(0, 2, (h, w, 1))
    p = tmp_path / "m.png"
    write_png(p, s, 1, 0, interlace)
    img = image_read(str(p))
    assert img.format == AB.FMT_MONOBLACK
    want = HostImage.from_array(s[:, :, 0].astype(bool), AB.FMT_MONOBLACK)
    assert np.array_equal(img.payload(), want.payload())


@pytest.mark.parametrize("depth,scale", [(2, 0x55), (4, 0x11)])
@pytest.mark.parametrize("interlace", [False, True])
def test_low_depth_gray_scaled(tmp_path, depth, scale, interlace):
    s = np.random.default_rng(depth).integers(0, 1 << depth, (11, 23, 1))
    p = tmp_path / "g.png"
    write_png(p, s, depth, 0, interlace)
    img = image_read(str(p))
    assert img.format == AB.FMT_GRAY8
    assert np.array_equal(img.payload(), (s[:, :, 0] * scale).astype(np.uint8))


@pytest.mark.parametrize("depth", [1, 2, 4, 8])
@pytest.mark.parametrize("interlace", [False, True])
def test_palette_to_rgb(tmp_path, depth, interlace):
    rng = np.random.default_rng(depth)
    npal = min(1 << depth, 200)
    plte = rng.integers(0, 256, (npal, 3))
    s = rng.integers(0, 1 << depth, (13, 29, 1))
    p = tmp_path / "p.png"
    write_png(p, s, depth, 3, interlace, plte=plte)
    img = image_read(str(p))
    assert img.format == AB.FMT_RGB24
    full = np.zeros((256, 3), dtype=np.uint8)  # past PLTE: black (FFmpeg's zeroed palette)
    full[:npal] = plte
    assert np.array_equal(img.payload(), full[s[:, :, 0]].reshape(13, 29 * 3))


def test_gray_trns_is_y400a(tmp_path):
    s = np.random.default_rng(3).integers(0, 4, (7, 9, 1)) * 60
    p = tmp_path / "t.png"
    write_png(p, s, 8, 0, trns=struct.pack(">H", 120))
    img = image_read(str(p))
    assert img.format == AB.FMT_Y400A
    want = np.stack([s[:, :, 0], np.where(s[:, :, 0] == 120, 0, 255)], axis=2)
    assert np.array_equal(img.payload(), want.reshape(7, 18).astype(np.uint8))


@pytest.mark.parametrize("depth,ctype,trns,what", [
    (16, 0, None, "unsupported pixel format"), (16, 2, None, "unsupported pixel format"),
    (8, 6, None, "unsupported pixel format"), (8, 2, b"\x00\x01\x00\x02\x00\x03",
                                              "unsupported pixel format")])
def test_unsupported_formats_fail_loudly(tmp_path, depth, ctype, trns, what):
    ch = {0: 1, 2: 3, 6: 4}[ctype]
    p = tmp_path / "u.png"
    write_png(p, np.zeros((3, 4, ch), dtype=np.int64), depth, ctype, trns=trns)
    with pytest.raises(UnpaperHipError, match=what):
        image_read(str(p))


def test_corrupt_and_truncated_fail_loudly(tmp_path):
    s = np.random.default_rng(9).integers(0, 256, (40, 50, 1))
    p = tmp_path / "ok.png"
    write_png(p, s, 8, 0)
    raw = open(p, "rb").read()
    trunc = tmp_path / "trunc.png"
    trunc.write_bytes(raw[: len(raw) // 2])
    with pytest.raises(UnpaperHipError):
        image_read(str(trunc))
    # a flipped byte inside the zlib stream: inflate or Adler-32 must catch it
    i = raw.index(b"IDAT") + 40
    bad = tmp_path / "bad.png"
    bad.write_bytes(raw[:i] + bytes([raw[i] ^ 0x5A]) + raw[i + 1:])
    with pytest.raises(UnpaperHipError):
        image_read(str(bad))
    # an invalid filter type byte
    rows = b"".join(b"\x07" + bytes(50) for _ in range(40))
    ft = tmp_path / "filt.png"
    ft.write_bytes(b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", 50, 40, 8, 0, 0, 0, 0))
                   + _chunk(b"IDAT", zlib.compress(rows)) + _chunk(b"IEND", b""))
    with pytest.raises(UnpaperHipError, match="filter"):
        image_read(str(ft))


def test_expect_mismatch_and_dispatch(tmp_path):
    L = load_library()
    s = np.random.default_rng(1).integers(0, 256, (6, 8, 1))
    p = tmp_path / "g.png"
    write_png(p, s, 8, 0)
    info = AB.PnmInfo()
    assert L.uphip_png_probe(str(p).encode(), C.byref(info)) == 0
    assert (info.width, info.height, info.format) == (8, 6, AB.FMT_GRAY8)
    wrong = AB.PnmInfo(8, 6, AB.FMT_RGB24)
    buf = np.zeros((6, 64), dtype=np.uint8)
    assert L.uphip_png_read(str(p).encode(), buf.ctypes.data, 64, C.byref(wrong)) != 0
    L.uphip_clear_error()
    assert L.uphip_png_read(str(p).encode(), buf.ctypes.data, 4, None) != 0  # linesize too small
    L.uphip_clear_error()
    # image_* picks the codec by signature: a PGM through the same entry point
    q = tmp_path / "g.pgm"
    pnm_write(str(q), HostImage.from_array(s[:, :, 0].astype(np.uint8), AB.FMT_GRAY8))
    a, b = image_read(str(p)), image_read(str(q))
    assert np.array_equal(a.payload(), b.payload())
    assert L.uphip_image_probe(b"/nonexistent.png", C.byref(info)) != 0
    L.uphip_clear_error()
