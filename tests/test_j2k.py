"""JPEG 2000 decode and lossless encode (the JP2 half of the
nvImageCodec peer: csrc/j2k.cpp host half, csrc/kernels_j2k.hip device half).

The reference hands .jp2/.j2k/.j2c files to nvImageCodec
(lib/decode_queue.c:53-71, 550) and writes .jp2 outputs with its lossless
parameters (lib/encode_queue.c:883-962).  nvImageCodec is absent here, so
parity is pinned to OpenJPEG 2.5 (PIL's JPEG 2000 codec), the decoder
nvImageCodec's CPU JPEG 2000 plugin also wraps:

- CPU: the decoder's host half + the device half replayed on the CPU
  (tests/c/j2k_emul.cpp: the device code-block decoder's lane code,
  j2k_t1_lane.h, in 64-block groups, and the same line functions; also the
  host code-block coder of j2k_t1.h) equals PIL's decode byte for
  byte on committed fixtures (tests/golden/j2k, tests/golden/make_j2k_fixtures.py)
  and a seeded matrix of encoder options (tiles, offsets, precincts,
  progression orders, code-block sizes, quality layers, 5/3 and 9/7, RCT/ICT);
  the encoder's packet data equal OpenJPEG's byte for byte and PIL decodes
  every file back to the input.
- GPU: uphip_jp2_read / _decode / image_read equal PIL's decode; the device
  encode equals the replayed encode byte for byte; the runner decodes JP2
  pages into its input slots and writes JP2 files through its sink.
"""
import ctypes as C
import glob
import io
import os

import numpy as np
import pytest
from PIL import Image

from unpaper_hip import ctypes_abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMUL = os.path.join(ROOT, "tests", "c", "_build", "libj2k_emul.so")
FIXTURES = os.path.join(ROOT, "tests", "golden", "j2k")


def _emul():
    from unpaper_hip.device import load_library
    load_library()  # the emulator links the library
    E = C.CDLL(EMUL)
    E.j2k_emulate.restype = C.c_int64
    E.j2k_emulate.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64, C.c_void_p]
    E.j2k_emulate_t1lane.restype = C.c_int64
    E.j2k_emulate_t1lane.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64, C.c_void_p]
    E.j2k_emulate_encode_lane.restype = C.c_int64
    E.j2k_emulate_encode_lane.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                          C.c_int64]
    E.j2k_emulate_encode.restype = C.c_int64
    E.j2k_emulate_encode.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                     C.c_int64]
    return E


def _err():
    from unpaper_hip.device import load_library
    L = load_library()
    e = L.uphip_last_error()
    L.uphip_clear_error()
    return e.decode() if e else None


def emulate_decode(data, lane=False):
    """The host half, then the code-blocks through j2k_t1.h's coder (or, with
    lane, the device decoder's lane code in 64-block groups) and the device
    half's line functions."""
    E = _emul()
    fn = E.j2k_emulate_t1lane if lane else E.j2k_emulate
    _err()  # a stale error from an earlier test in this worker must not name this one's
    info = (C.c_int32 * 3)()
    n = fn(data, len(data), None, 0, info)
    if n < 0:
        raise ValueError(_err())
    out = np.zeros(n, np.uint8)
    assert fn(data, len(data), out.ctypes.data, n, info) == n
    w, h, c = info
    return out.reshape(h, w, c) if c > 1 else out.reshape(h, w)


def emulate_encode(a, lane=False):
    """The device's forward transforms replayed, then the code-blocks through
    j2k_t1.h's host coder (or, with lane, the device encoder's lane code in
    64-block groups) and the host's packets."""
    E = _emul()
    fn = E.j2k_emulate_encode_lane if lane else E.j2k_emulate_encode
    a = np.ascontiguousarray(a)
    h, w = a.shape[:2]
    c = 1 if a.ndim == 2 else 3
    n = fn(a.ctypes.data, w, h, c, None, 0)
    assert n > 0, _err()
    out = np.zeros(n, np.uint8)
    assert fn(a.ctypes.data, w, h, c, out.ctypes.data, n) == n
    return out.tobytes()


def pil_save(a, **kw):
    b = io.BytesIO()
    Image.fromarray(a).save(b, "JPEG2000", **kw)
    return b.getvalue()


def pil_decode(data):
    return np.asarray(Image.open(io.BytesIO(data)))


def page(w, h, seed, rgb=False):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    g = np.full((h, w), 255, np.uint8)
    for r in range(3, h - 6, 9):
        for c0 in range(2, w - 10, 13):
            if rng.random() < 0.6:
                g[r:r + 5, c0:c0 + rng.integers(2, 10)] = rng.integers(0, 70)
    g[: h // 5] = ((x * 3 + y * 7) % 256)[: h // 5]
    g[h // 2:h // 2 + h // 6, w // 3:2 * w // 3] = rng.integers(0, 256, (h // 6, 2 * w // 3 - w // 3))
    if not rgb:
        return g
    return np.stack([g, np.roll(g, 7, 1), np.maximum(g, 90)], 2)


# encoder options the decoder must take (PIL / OpenJPEG names)
OPTIONS = [
    {},
    {"num_resolutions": 1},
    {"num_resolutions": 2, "codeblock_size": (4, 4)},
    {"tile_size": (32, 48)},
    {"tile_size": (40, 40), "tile_offset": (3, 5), "offset": (7, 11)},
    {"progression": "RLCP", "quality_mode": "rates", "quality_layers": [30, 10, 3]},
    {"progression": "RPCL", "precinct_size": (32, 32)},
    {"progression": "PCRL", "precinct_size": (16, 16), "codeblock_size": (8, 16)},
    {"progression": "CPRL", "tile_size": (64, 64), "precinct_size": (32, 64)},
    {"irreversible": True},
    {"irreversible": True, "quality_mode": "rates", "quality_layers": [50, 12]},
    {"irreversible": True, "tile_size": (48, 32), "progression": "RPCL"},
    {"codeblock_size": (64, 16), "plt": True},
    {"no_jp2": True},
]


# ---------------------------------------------------------------------------
# CPU: the restated decoder (host half + replayed device half) against PIL
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("name", sorted(os.path.basename(p) for p in
                                        glob.glob(os.path.join(FIXTURES, "*.j*"))))
@pytest.mark.parametrize("lane", [False, True])
def test_fixtures_decode_as_openjpeg(name, lane):
    data = open(os.path.join(FIXTURES, name), "rb").read()
    exp = np.load(os.path.join(FIXTURES, name.rsplit(".", 1)[0] + ".npy"))
    got = emulate_decode(data, lane)
    assert got.shape == exp.shape and (got == exp).all(), name


@pytest.mark.parametrize("opt", range(len(OPTIONS)))
@pytest.mark.parametrize("rgb,mct", [(False, 0), (True, 0), (True, 1)])
def test_decode_matches_openjpeg(opt, rgb, mct):
    kw = dict(OPTIONS[opt])
    if rgb:
        kw["mct"] = mct
    for w, h in ((83, 67), (128, 96), (5, 3)):
        if "tile_size" in kw and (w < 40 or h < 40):
            continue
        a = page(w, h, opt * 7 + w, rgb)
        data = pil_save(a, **kw)
        exp = pil_decode(data)
        for lane in (False, True):
            got = emulate_decode(data, lane)
            assert got.shape == exp.shape and (got == exp).all(), (kw, w, h, lane)
        if not kw.get("irreversible") and "quality_layers" not in kw:
            assert (got == a).all()  # lossless


def test_pair_lifting_equals_sequential_lifting():
    """The device kernels lift one output pair a thread over a window of the
    line's symmetric extension (j2k_dwt.h idwt_pair / fdwt53_pair); against
    the in-place sequential lifting for every length 1..200 and both
    parities: 5/3 both ways, 9/7 inverse, bit for bit."""
    E = _emul()
    E.j2k_dwt_check.restype = C.c_int64
    E.j2k_dwt_check.argtypes = [C.c_int, C.c_uint32]
    for seed in (1, 7, 1234):
        assert E.j2k_dwt_check(200, seed) == 0


def test_decode_refuses_what_it_does_not_take(tmp_path):
    a16 = (np.arange(24 * 20, dtype=np.uint16).reshape(20, 24) * 97)
    data16 = pil_save(a16)  # 16-bit precision
    with pytest.raises(ValueError):
        emulate_decode(data16)
    la = np.stack([page(30, 20, 1), np.full((20, 30), 255, np.uint8)], 2)
    b = io.BytesIO()
    Image.fromarray(la, "LA").save(b, "JPEG2000")
    with pytest.raises(ValueError, match="component"):
        emulate_decode(b.getvalue())
    for junk in (b"", b"\x00\x00\x00\x0cjP  \r\n\x87\n", b"\xff\x4f\xff\x51" + b"\x00" * 40,
                 os.urandom(300)):
        with pytest.raises(ValueError):
            emulate_decode(junk)


def test_decode_truncated_and_corrupt_files_do_not_crash():
    """Cut or bit-flipped files either fail with an error or decode to an
    image of the header's geometry; none may crash (the sanitizer run covers
    the same under ASan)."""
    a = page(70, 50, 3, True)
    data = pil_save(a, mct=1, quality_mode="rates", quality_layers=[20, 5])
    rng = np.random.default_rng(0)
    for cut in range(0, len(data), max(1, len(data) // 23)):
        try:
            got = emulate_decode(data[:cut])
            assert got.shape == a.shape
        except ValueError:
            pass
    for k in range(40):
        d = bytearray(data)
        i = int(rng.integers(0, len(d)))
        d[i] ^= int(rng.integers(1, 256))
        try:
            emulate_decode(bytes(d))
        except ValueError:
            pass


def test_probe_and_image_probe(tmp_path):
    from unpaper_hip.device import load_library
    L = load_library()
    for name, fmt in (("gray.jp2", A.FMT_GRAY8), ("rgb_mct.jp2", A.FMT_RGB24),
                      ("tiled_rpcl.j2k", A.FMT_GRAY8)):
        path = os.path.join(FIXTURES, name).encode()
        for fn in (L.uphip_jp2_probe, L.uphip_image_probe):
            info = A.PnmInfo()
            assert fn(path, C.byref(info)) == 0, _err()
            assert (info.width, info.height, info.format) == (77, 61, fmt)
    info = A.PnmInfo()
    assert L.uphip_jp2_probe(os.path.join(FIXTURES, "gray.npy").encode(), C.byref(info)) == -1
    assert _err()


def test_entropy_decode_host_half():
    from unpaper_hip.device import load_library
    L = load_library()
    data = open(os.path.join(FIXTURES, "gray.jp2"), "rb").read()
    info = A.PnmInfo()
    n = L.uphip_jp2_entropy_decode(data, len(data), None, 0, C.byref(info))
    assert n == 77 * 61 * 4 and (info.width, info.height) == (77, 61)
    buf = np.zeros(n // 4, np.int32)
    assert L.uphip_jp2_entropy_decode(data, len(data), buf.ctypes.data, n, C.byref(info)) == n
    assert buf.any()


# ---------------------------------------------------------------------------
# CPU: the lossless encoder (device transforms replayed) against OpenJPEG
# ---------------------------------------------------------------------------

def _body(f):
    return f[f.index(b"\xff\x93") + 2:]


@pytest.mark.parametrize("w,h", [(1, 1), (1, 13), (17, 1), (2, 2), (37, 53), (64, 64),
                                 (65, 129), (300, 211)])
@pytest.mark.parametrize("rgb", [False, True])
def test_encode_is_lossless_and_matches_openjpeg(w, h, rgb):
    a = page(w, h, w * 31 + h, rgb) if w > 8 and h > 8 else \
        np.random.default_rng(w + h).integers(0, 256, (h, w, 3) if rgb else (h, w)).astype(np.uint8)
    f = emulate_encode(a)
    assert emulate_encode(a, lane=True) == f  # the device encoder's lane code
    assert f[:12] == b"\x00\x00\x00\x0cjP  \r\n\x87\n"
    assert (pil_decode(f) == a).all()
    assert (emulate_decode(f) == a).all()
    ref = pil_save(a, mct=1) if rgb else pil_save(a)
    assert _body(f) == _body(ref)  # OpenJPEG's packets, byte for byte


def test_encode_uniform_and_extreme_pages():
    for a in (np.zeros((40, 50), np.uint8), np.full((40, 50, 3), 255, np.uint8),
              np.tile(np.array([0, 255], np.uint8), (33, 20))):
        f = emulate_encode(a)
        assert (pil_decode(f) == a).all()
        ref = pil_save(a, mct=1) if a.ndim == 3 else pil_save(a)
        assert _body(f) == _body(ref)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------

def _device_image(a, pad=0):
    from unpaper_hip.pipeline import DeviceBuffer
    from unpaper_hip.device import load_library
    L = load_library()
    h = a.shape[0]
    row = a.shape[1] * (1 if a.ndim == 2 else 3)
    pitch = row + pad
    host = np.zeros((h, pitch), np.uint8)
    host[:, :row] = a.reshape(h, row)
    d = DeviceBuffer(pitch * h)
    assert L.uphip_memcpy_htod(d.ptr, host.ctypes.data, pitch * h) == 0
    return d, pitch


@pytest.mark.gpu
def test_device_read_matches_openjpeg(hip, tmp_path):
    from unpaper_hip.pipeline import image_read
    for opt in range(len(OPTIONS)):
        for rgb in (False, True):
            kw = dict(OPTIONS[opt])
            if rgb:
                kw["mct"] = 1
            a = page(131, 97, opt, rgb)
            p = tmp_path / ("x%d_%d.%s" % (opt, rgb, "j2k" if kw.get("no_jp2") else "jp2"))
            p.write_bytes(pil_save(a, **kw))
            got = image_read(str(p))
            exp = pil_decode(p.read_bytes())
            arr = got.to_gray() if not rgb else got.to_rgb()
            assert arr.shape == exp.shape and (arr == exp).all(), kw


@pytest.mark.gpu
def test_device_decode_into_device_memory(hip):
    from unpaper_hip.device import load_library
    L = load_library()
    for name in sorted(glob.glob(os.path.join(FIXTURES, "*.j*"))):
        data = open(name, "rb").read()
        exp = np.load(name.rsplit(".", 1)[0] + ".npy")
        h, w = exp.shape[:2]
        row = w * (1 if exp.ndim == 2 else 3)
        pitch = (row + 300) // 256 * 256 + 256
        from unpaper_hip.pipeline import DeviceBuffer
        d = DeviceBuffer(pitch * h)
        try:
            info = A.PnmInfo()
            assert L.uphip_jp2_decode(data, len(data), d.ptr, pitch, C.byref(info)) == 0, _err()
            assert (info.width, info.height) == (w, h)
            host = np.zeros((h, pitch), np.uint8)
            assert L.uphip_memcpy_dtoh(host.ctypes.data, d.ptr, pitch * h) == 0
            got = host[:, :row].reshape(exp.shape)
            assert (got == exp).all(), name
            bad = A.PnmInfo(w + 1, h, info.format)  # expected geometry mismatch
            assert L.uphip_jp2_decode(data, len(data), d.ptr, pitch, C.byref(bad)) == -1
            assert _err()
        finally:
            d.close()


@pytest.mark.gpu
def test_device_decode_a4_pages(hip, tmp_path):
    """An A4 300 dpi page (2480 x 3508), gray and RGB, lossless and 9/7
    with layers, several tiles: equal to OpenJPEG."""
    from unpaper_hip.pipeline import image_read, synth_page_host
    g = synth_page_host(2480, 3508, 5)
    rgb = np.stack([g, np.roll(g, 5, 1), np.maximum(g, 30)], 2)
    for a, kw in ((g, {}), (rgb, {"mct": 1, "tile_size": (1024, 1024)}),
                  (g, {"irreversible": True, "quality_mode": "rates", "quality_layers": [40]})):
        p = tmp_path / "a4.jp2"
        p.write_bytes(pil_save(a, **kw))
        got = image_read(str(p))
        arr = got.to_gray() if a.ndim == 2 else got.to_rgb()
        assert (arr == pil_decode(p.read_bytes())).all(), kw


@pytest.mark.gpu
@pytest.mark.parametrize("rgb", [False, True])
def test_device_encode_equals_replay(hip, rgb):
    from unpaper_hip.pipeline import jp2_encode
    for w, h in ((1, 1), (33, 17), (250, 131), (2480, 3508)):
        a = page(w, h, w + h, rgb) if w > 8 else np.full((h, w, 3) if rgb else (h, w), 9, np.uint8)
        for pad in (0, 256 - (a.shape[1] * (3 if rgb else 1)) % 256):
            d, pitch = _device_image(a, pad)
            try:
                f = jp2_encode(d.ptr, pitch, w, h, A.FMT_RGB24 if rgb else A.FMT_GRAY8)
            finally:
                d.close()
            assert f == emulate_encode(a), (w, h, pad)
            if w * h < 10 ** 6:
                assert (pil_decode(f) == a).all()


@pytest.mark.gpu
def test_device_encode_errors(hip):
    from unpaper_hip.device import load_library
    L = load_library()
    a = page(40, 30, 1)
    d, pitch = _device_image(a)
    try:
        for args in ((pitch, 40, 30, A.FMT_Y400A), (10, 40, 30, A.FMT_GRAY8),
                     (pitch, 0, 30, A.FMT_GRAY8)):
            assert L.uphip_jp2_encode(d.ptr, *args, None, 0) == -1, args
            assert _err()
        n = L.uphip_jp2_encode(d.ptr, pitch, 40, 30, A.FMT_GRAY8, None, 0)
        assert n > 0
        small = np.zeros(n - 1, np.uint8)
        assert L.uphip_jp2_encode(d.ptr, pitch, 40, 30, A.FMT_GRAY8, small.ctypes.data, n - 1) == n
        assert not small.any()  # nothing copied when the capacity is short
    finally:
        d.close()


@pytest.mark.gpu
def test_runner_jp2_sources_and_sink(hip, oracle, tmp_path):
    """The decode queue's JP2 branch and the encode queue's .jp2 branch
    through the runner: a chunk mixing JP2 (lossless, 9/7, tiled), JPEG and
    PNM pages of one RGB24 geometry decodes each on the slot's stream; the
    sheets equal the oracle on OpenJPEG's decode, and the JP2 sink's files
    decode (PIL) to those same sheets."""
    from unpaper_hip.hostimage import HostImage
    from unpaper_hip.pipeline import Runner, sink_jp2, sink_pnm, source_pnm, pnm_write, pnm_read
    w, h = 300, 420
    opts = oracle.default_options()
    paths, pages = [], []
    for i in range(6):
        a = page(w, h, 50 + i, True)
        if i == 2:
            q = str(tmp_path / ("p%d.ppm" % i))
            pnm_write(q, HostImage.from_array(a, A.FMT_RGB24))
            px = a
        elif i == 4:
            q = str(tmp_path / ("p%d.jpg" % i))
            Image.fromarray(a).save(q, "JPEG", quality=90)
            px = np.asarray(Image.open(q))
        else:
            q = str(tmp_path / ("p%d.jp2" % i))
            kw = [{"mct": 1}, {"irreversible": True, "mct": 1}, None, {"tile_size": (128, 128)},
                  None, {"progression": "RPCL", "quality_mode": "rates",
                         "quality_layers": [30]}][i]
            open(q, "wb").write(pil_save(a, **kw))
            px = pil_decode(open(q, "rb").read())
        paths.append(q)
        pages.append(HostImage.from_array(np.ascontiguousarray(px), A.FMT_RGB24))
    exp = []
    for p in pages:
        sheet, fmt, _ = oracle.process_sheet(opts, [p])
        exp.append(oracle.convert_for_save(sheet, fmt))
    r = Runner(opts, 4, w, h, A.FMT_RGB24, devices=(0,), streams=2, host_threads=3)
    try:
        failed, err = r.run_host(len(paths), source_pnm(paths), sink_pnm(str(tmp_path / "o%02d.ppm")))
        assert failed == 0, err
        failed, err = r.run_host(len(paths), source_pnm(paths), sink_jp2(str(tmp_path / "o%02d.jp2")))
        assert failed == 0, err
    finally:
        r.close()
    for i in range(len(paths)):
        got = pnm_read(str(tmp_path / ("o%02d.ppm" % i)))
        assert (got.payload() == exp[i].payload()).all(), (i, paths[i])
        j = pil_decode(open(tmp_path / ("o%02d.jp2" % i), "rb").read())
        assert (j == got.to_rgb()).all(), i


def test_sink_jp2_argument_checks():
    from unpaper_hip.device import load_library
    L = load_library()
    assert not L.uphip_sink_jp2(b"x%s.jp2", 0)
    assert _err()
    k = L.uphip_sink_jp2(b"x%04d.jp2", 0)
    assert k
    L.uphip_sink_destroy(k)
