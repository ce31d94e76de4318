"""GPU parity of the filters and rotation detection (filters.c / deskew.c
peers): HIP == oracle bit for bit.  The small hand-made scenes restate the
reference's own unit tests (tests/cuda_filters_test.c:42-383,
tests/cuda_deskew_test.c:18-40); the synthetic pages exercise the default
parameters, order-dependent cases (clustered specks, edge-zone quirks, wipe
feedback on colour tiles, flood fills) and odd geometries."""
import math

import numpy as np
import pytest

from unpaper_hip import ctypes_abi as A
from unpaper_hip.hostimage import HostImage
from helpers import FORMATS, assert_same, make_image

pytestmark = pytest.mark.gpu

WHITE, BLACK = A.Pixel(255, 255, 255), A.Pixel(0, 0, 0)


def blank(w, h, fmt, thr):
    shape = {A.FMT_RGB24: (h, w, 3), A.FMT_Y400A: (h, w, 2)}.get(fmt, (h, w))
    return HostImage.from_array(np.full(shape, 255, np.uint8), fmt, abs_black_threshold=thr)


def put(oracle, h, x, y, px):
    oracle.wipe_rectangle(h, A.rect(x, y, x, y), px)


def both(hip, oracle, h, op_hip, op_oracle):
    d = hip.upload(h)
    op_hip(d)
    op_oracle(h)
    assert_same(d.to_host(), h)


# ---------------------------------------------------------------- noisefilter
def scene_noise(oracle, h):          # cuda_filters_test.c:42-54
    put(oracle, h, 5, 5, BLACK)
    oracle.wipe_rectangle(h, A.rect(15, 10, 17, 12), BLACK)


def scene_noise_diag(oracle, h):     # cuda_filters_test.c:56-75
    for i in range(4):
        put(oracle, h, 2 + i, 2 + i, BLACK)
    for dx, dy in [(0, 0), (1, 0), (-1, 0), (0, 1), (0, -1)]:
        put(oracle, h, 12 + dx, 12 + dy, BLACK)
    put(oracle, h, 24, 6, BLACK)
    put(oracle, h, 25, 6, BLACK)


@pytest.mark.parametrize("scene,fmt,size,thr,intensity,white", [
    (scene_noise, A.FMT_GRAY8, (32, 24), 64, 2, 200),
    (scene_noise_diag, A.FMT_GRAY8, (32, 24), 64, 4, 200),
    (scene_noise_diag, A.FMT_GRAY8, (32, 24), 64, 3, 200),
    (scene_noise, A.FMT_Y400A, (20, 16), 64, 3, 180),
])
def test_noisefilter_reference_scenes(hip, oracle, scene, fmt, size, thr, intensity, white):
    h = blank(*size, fmt, thr)
    scene(oracle, h)
    both(hip, oracle, h, lambda d: hip.noisefilter(d, intensity, white),
         lambda o: oracle.noisefilter(o, intensity, white))


def test_noisefilter_rgb_scene(hip, oracle):  # cuda_filters_test.c:77-90
    h = blank(32, 24, A.FMT_RGB24, 64)
    put(oracle, h, 4, 4, A.Pixel(30, 0, 0))
    put(oracle, h, 5, 4, A.Pixel(28, 0, 0))
    oracle.wipe_rectangle(h, A.rect(14, 10, 16, 12), A.Pixel(20, 40, 60))
    both(hip, oracle, h, lambda d: hip.noisefilter(d, 2, 200),
         lambda o: oracle.noisefilter(o, 2, 200))


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("size,seed,specks", [((300, 200), 1, 400), ((640, 480), 2, 3000),
                                              ((129, 257), 3, 800), ((1000, 700), 4, 6000)])
@pytest.mark.parametrize("intensity", [4, 2, 6])
def test_noisefilter_pages(hip, oracle, fmt, size, seed, specks, intensity):
    # dense specks -> many clustered (sequentially resolved) components; specks
    # touch the left/top edge -> the unsigned-loop quirk zone
    h = make_image(*size, fmt, seed=seed, specks=specks, margin=0)
    both(hip, oracle, h, lambda d: hip.noisefilter(d, intensity, 229),
         lambda o: oracle.noisefilter(o, intensity, 229))


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24])
@pytest.mark.parametrize("density,intensity", [(0.12, 4), (0.3, 4), (0.3, 2), (0.55, 3)])
def test_noisefilter_dense_salt(hip, oracle, fmt, density, intensity):
    # so many small components per 64x64 tile that the classify kernel's LDS
    # work lists overflow and it takes its row-loop path
    rng = np.random.default_rng(int(density * 100) + intensity)
    g = np.where(rng.random((230, 301)) < density, rng.integers(0, 200, (230, 301)), 255)
    g = g.astype(np.uint8)
    if fmt == A.FMT_RGB24:
        h = HostImage.from_array(np.repeat(g[:, :, None], 3, axis=2), fmt)
    else:
        h = HostImage.from_array(g, fmt)
    both(hip, oracle, h, lambda d: hip.noisefilter(d, intensity, 229),
         lambda o: oracle.noisefilter(o, intensity, 229))


def test_noisefilter_edge_quirk(hip, oracle):
    # components hugging x < level / y < level-1, where the reference's ring
    # loops skip whole rows (int32 vs uint32 comparison)
    g = np.full((40, 50), 255, np.uint8)
    for (x, y) in [(0, 0), (1, 0), (0, 5), (1, 6), (2, 10), (0, 20), (3, 1), (10, 0), (11, 1),
                   (20, 2), (21, 2), (22, 2), (2, 30), (2, 31), (3, 31), (4, 31), (1, 32)]:
        g[y, x] = 0
    h = HostImage.from_array(g, A.FMT_GRAY8)
    both(hip, oracle, h, lambda d: hip.noisefilter(d, 4, 229),
         lambda o: oracle.noisefilter(o, 4, 229))


def noisy_scan(w, h, page, specks, seed, quality=75, border=True, dashes=True):
    """A synthetic page made to look like a poor scan: clustered 1-px specks
    (sequentially resolved components), a ragged dark left border (the
    edge zone; its interior is the no-op triggers k_noise_classify drops), a
    dashed rule in the top zone (one row of several hundred triggers), all
    through a JPEG round trip (compression noise)."""
    import io
    from PIL import Image
    from unpaper_hip.pipeline import synth_page_host
    g = synth_page_host(w, h, page).copy()
    rng = np.random.default_rng(seed)
    ys, xs = rng.integers(0, h, specks), rng.integers(0, w, specks)
    g[ys, xs] = rng.integers(0, 120, specks)
    if border:
        edge = 20 + rng.integers(0, 12, h)
        for y in range(h):
            g[y, :edge[y]] = 30
    if dashes:
        g[3, 40::2] = 0
        g[9, 100::3] = 10
    b = io.BytesIO()
    Image.fromarray(g).save(b, "JPEG", quality=quality)
    return np.asarray(Image.open(io.BytesIO(b.getvalue()))).copy()


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24])
@pytest.mark.parametrize("specks,intensity", [(40000, 4), (40000, 2), (6000, 4), (800, 3), (800, 4)])
def test_noisefilter_group_caps(hip, oracle, fmt, specks, intensity):
    # 40000 / 6000 specks: more than 4096 sequential triggers (k_noise_group's
    # global layout); 800: within its LDS layout; all with rows of more than
    # 256 triggers (the dashed rules: the block-wide bucket sort)
    g = noisy_scan(1240, 1754, 3, specks, specks + intensity)
    h = HostImage.from_array(np.repeat(g[:, :, None], 3, axis=2) if fmt == A.FMT_RGB24 else g, fmt)
    both(hip, oracle, h, lambda d: hip.noisefilter(d, intensity, 229),
         lambda o: oracle.noisefilter(o, intensity, 229))


def test_noisefilter_border_quirk_strip(hip, oracle):
    # a solid border band with thin spurs reaching into the quirk strip
    # (x < 7, y < 6): the no-op trigger test must leave those in the sequence
    g = np.full((300, 400), 255, np.uint8)
    g[:, :25] = 0
    g[:40, :] = 0
    for y in range(45, 300, 7):
        g[y, 25:25 + (y % 11)] = 0      # spurs off the band's edge
        g[y + 1, 3] = 255               # notches inside the quirk strip
    g[50:60, 0:2] = 255
    g[2, 100:300:2] = 255
    h = HostImage.from_array(g, A.FMT_GRAY8)
    both(hip, oracle, h, lambda d: hip.noisefilter(d, 4, 229),
         lambda o: oracle.noisefilter(o, 4, 229))


# ---------------------------------------------------------------- grayfilter
def test_grayfilter_reference_scene(hip, oracle):  # cuda_filters_test.c:296-331
    h = blank(8, 8, A.FMT_GRAY8, 50)
    oracle.wipe_rectangle(h, A.rect(0, 0, 3, 3), A.Pixel(150, 150, 150))
    oracle.wipe_rectangle(h, A.rect(4, 0, 7, 3), A.Pixel(80, 80, 80))
    p = A.GrayfilterParameters(A.RectangleSize(4, 4), A.Delta(4, 4), 127)
    both(hip, oracle, h, lambda d: hip.grayfilter(d, p), lambda o: oracle.grayfilter(o, p))


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("size", [(300, 200), (1001, 777), (50, 50), (7, 3)])
@pytest.mark.parametrize("params", [((50, 50), (20, 20), 127), ((30, 20), (15, 8), 127),
                                    ((50, 50), (20, 20), 200), ((13, 7), (5, 3), 60)])
def test_grayfilter_pages(hip, oracle, fmt, size, params):
    h = make_image(*size, fmt, seed=5)
    p = A.GrayfilterParameters(A.RectangleSize(*params[0]), A.Delta(*params[1]), params[2])
    both(hip, oracle, h, lambda d: hip.grayfilter(d, p), lambda o: oracle.grayfilter(o, p))


@pytest.mark.parametrize("black", [40, 100, 170])
def test_grayfilter_feedback_rgb(hip, oracle, black):
    # saturated colour blocks: gray > black threshold but min(rgb) tiny, so a
    # tile fails on the original image and passes once earlier tiles are wiped
    rng = np.random.default_rng(7)
    rgb = np.full((260, 330, 3), 255, np.uint8)
    for _ in range(60):
        x, y = int(rng.integers(0, 320)), int(rng.integers(0, 250))
        rgb[y:y + int(rng.integers(3, 30)), x:x + int(rng.integers(3, 30))] = \
            [int(rng.integers(200, 256)), int(rng.integers(200, 256)), int(rng.integers(0, 30))]
    h = HostImage.from_array(rgb, A.FMT_RGB24, abs_black_threshold=black)
    for thr in (127, 160, 90):
        p = A.GrayfilterParameters(A.RectangleSize(50, 50), A.Delta(20, 20), thr)
        hh = h.copy()
        both(hip, oracle, hh, lambda d: hip.grayfilter(d, p), lambda o: oracle.grayfilter(o, p))


# ---------------------------------------------------------------- blurfilter
def test_blurfilter_reference_scene(hip, oracle):  # cuda_filters_test.c:337-383
    h = blank(16, 16, A.FMT_GRAY8, 64)
    for (x, y) in [(1, 5), (2, 5), (1, 6)]:
        put(oracle, h, x, y, BLACK)
    oracle.wipe_rectangle(h, A.rect(8, 4, 11, 7), BLACK)
    p = A.BlurfilterParameters(A.RectangleSize(4, 4), A.Delta(2, 2), 0.1)
    both(hip, oracle, h, lambda d: hip.blurfilter(d, p, 200),
         lambda o: oracle.blurfilter(o, p, 200))


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("size", [(2480 // 4, 3508 // 4), (1001, 777), (99, 300), (100, 100)])
@pytest.mark.parametrize("params", [((100, 100), (50, 50), 0.01), ((40, 30), (15, 20), 0.05),
                                    ((64, 64), (64, 13), 0.2)])
def test_blurfilter_pages(hip, oracle, fmt, size, params):
    h = make_image(*size, fmt, seed=6, specks=300)
    p = A.BlurfilterParameters(A.RectangleSize(*params[0]), A.Delta(*params[1]), params[2])
    both(hip, oracle, h, lambda d: hip.blurfilter(d, p, 229),
         lambda o: oracle.blurfilter(o, p, 229))


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24])
@pytest.mark.parametrize("width", [1320, 2000, 3960, 4480, 4520])
def test_blurfilter_wide_rows(hip, oracle, fmt, width):
    # rows of 33 .. 112 blocks take the chunked scalar resolver (C4's 99),
    # 113 the generic one
    h = make_image(width, 300, fmt, seed=7, specks=600)
    for params in (((40, 30), (15, 20), 0.05), ((40, 40), (40, 10), 0.3)):
        p = A.BlurfilterParameters(A.RectangleSize(*params[0]), A.Delta(*params[1]), params[2])
        both(hip, oracle, h.copy(), lambda d: hip.blurfilter(d, p, 229),
             lambda o: oracle.blurfilter(o, p, 229))


# ---------------------------------------------------------------- blackfilter
def black_params(oracle, size=(20, 20), step=(5, 5), depth=(500, 500), thr=242, intensity=20,
                 direction=(True, True), exclusions=()):
    p = oracle.default_options().blackfilter_parameters
    p.scan_size = A.RectangleSize(*size)
    p.scan_step = A.Delta(*step)
    p.scan_depth.horizontal, p.scan_depth.vertical = depth
    p.abs_threshold = thr
    p.intensity = intensity
    p.scan_direction = A.Direction(*direction)
    p.exclusions_count = len(exclusions)
    for i, e in enumerate(exclusions):
        p.exclusions[i] = A.rect(*e)
    return p


def test_blackfilter_reference_scene(hip, oracle):  # cuda_filters_test.c:249-290
    h = blank(32, 24, A.FMT_GRAY8, 128)
    oracle.wipe_rectangle(h, A.rect(8, 0, 11, 23), BLACK)
    p = black_params(oracle, (4, 4), (2, 2), (32, 24), int(255 * np.float32(0.9)), 2)
    both(hip, oracle, h, lambda d: hip.blackfilter(d, p), lambda o: oracle.blackfilter(o, p))


def band_page(w, h, fmt, band, seed, noise=True):
    rng = np.random.default_rng(seed)
    g = make_image(w, h, A.FMT_GRAY8, seed=seed).to_gray()
    x0, x1, y0, y1 = band
    g[y0:y1, x0:x1] = rng.integers(0, 11, size=(y1 - y0, x1 - x0)) if noise else 0
    if fmt == A.FMT_GRAY8:
        return HostImage.from_array(g, fmt)
    if fmt == A.FMT_RGB24:
        return HostImage.from_array(np.repeat(g[:, :, None], 3, axis=2), fmt)
    if fmt == A.FMT_Y400A:
        return HostImage.from_array(np.stack([g, np.full_like(g, 255)], axis=2), fmt)
    return HostImage.from_array(g >= 128, fmt)      # 1-bit: white where gray >= 128


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("band", [(0, 40, 0, 700), (0, 600, 0, 25), (560, 600, 100, 300),
                                  (0, 30, 200, 400)])
def test_blackfilter_bands(hip, oracle, fmt, band):
    h = band_page(600, 700, fmt, band, seed=8)
    p = black_params(oracle, exclusions=[(150, 175, 449, 524)])
    both(hip, oracle, h, lambda d: hip.blackfilter(d, p), lambda o: oracle.blackfilter(o, p))


@pytest.mark.parametrize("intensity", [20, 1, 3])
@pytest.mark.parametrize("size", [(300, 400), (123, 77)])
def test_blackfilter_irregular(hip, oracle, intensity, size):
    # dark blobs with holes, gaps and stray strokes: the fill order matters
    rng = np.random.default_rng(intensity + size[0])
    w, hh = size
    g = np.full((hh, w), 255, np.uint8)
    g[:, :12] = rng.integers(0, 40, size=(hh, 12))
    for _ in range(40):
        y, x = int(rng.integers(0, hh)), int(rng.integers(0, 30))
        g[y:y + int(rng.integers(1, 5)), x:x + int(rng.integers(1, 25))] = rng.integers(0, 200)
    g[rng.random((hh, w)) < 0.02] = 0
    h = HostImage.from_array(g, A.FMT_GRAY8)
    p = black_params(oracle, intensity=intensity, depth=(100, 100))
    both(hip, oracle, h, lambda d: hip.blackfilter(d, p), lambda o: oracle.blackfilter(o, p))


def as_format(g, fmt, rng, thr=None):
    """A gray array in `fmt`: RGB24 channels tinted apart (as the C4 pages),
    Y400A with a random alpha."""
    kw = {} if thr is None else {"abs_black_threshold": thr}
    if fmt == A.FMT_RGB24:
        t = rng.integers(0, 9, size=3)
        rgb = np.stack([np.maximum(g.astype(int) - int(t[c]), 0) for c in range(3)], axis=2)
        return HostImage.from_array(rgb.astype(np.uint8), fmt, **kw)
    if fmt == A.FMT_Y400A:
        a = rng.integers(0, 256, size=g.shape, dtype=np.uint8)
        return HostImage.from_array(np.stack([g, a], axis=2), fmt, **kw)
    return HostImage.from_array(g, fmt, **kw)


def speck_page(w, h, density, seed, band=(5, 25)):
    """A dark band for the bars to find, and dark specks a fill line can
    reach through up to intensity-1 light pixels: the pattern of the heavy
    C4 sheets, where one fill percolates through the page's salt specks."""
    rng = np.random.default_rng(seed)
    g = np.full((h, w), 255, np.uint8)
    g[:, band[0]:band[1]] = rng.integers(0, 12, size=(h, band[1] - band[0]))
    m = rng.random((h, w)) < density
    g[m] = rng.integers(0, 60, size=int(m.sum()))
    return g, rng


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24, A.FMT_Y400A])
@pytest.mark.parametrize("density,intensity", [(0.08, 20), (0.2, 6), (0.1, 30)])  # 383, 687, 3818 frames
def test_blackfilter_percolation(hip, oracle, fmt, density, intensity):
    # thousands of short frames, most with several matching neighbours: the
    # replay's resume-past-the-windows rule and its stack run every path
    g, rng = speck_page(400, 300, density, seed=int(density * 1000) + intensity)
    h = as_format(g, fmt, rng)
    p = black_params(oracle, intensity=intensity, depth=(100, 100))
    both(hip, oracle, h, lambda d: hip.blackfilter(d, p), lambda o: oracle.blackfilter(o, p))


@pytest.mark.parametrize("intensity", [0, 63, 64, 65, 1000])
def test_blackfilter_intensity_edges(hip, oracle, intensity):
    # 0: the counter is 0 after the first position whatever it holds (every
    # line empty); 63 / 64 / 65: the window's run test switches from the
    # in-window smear to the cross-window carry; 1000: lines run to the edge
    g, rng = speck_page(300, 200, 0.05, seed=intensity)
    h = as_format(g, A.FMT_GRAY8, rng)
    p = black_params(oracle, intensity=intensity, depth=(100, 100))
    both(hip, oracle, h, lambda d: hip.blackfilter(d, p), lambda o: oracle.blackfilter(o, p))


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24])
def test_blackfilter_long_lines(hip, oracle, fmt):
    # fill lines over 1024 positions (several round trips a line) and
    # neighbour runs over 512 (several check windows), in both directions
    g, rng = speck_page(2600, 1300, 0.01, seed=7, band=(0, 30))
    g[600:606, :] = rng.integers(0, 20, size=(6, 2600))   # a row band across the page
    g[:, 1800:1804] = rng.integers(0, 20, size=(1300, 4))  # a column band down it
    h = as_format(g, fmt, rng)
    p = black_params(oracle, intensity=20, depth=(200, 200))
    both(hip, oracle, h, lambda d: hip.blackfilter(d, p), lambda o: oracle.blackfilter(o, p))


@pytest.mark.parametrize("thr", [0, 30, 254])
def test_blackfilter_mask_max(hip, oracle, thr):
    # the image's abs_black_threshold is the fill's match bound (fill.c:85):
    # 0 matches only black, 254 everything but white
    g, rng = speck_page(300, 200, 0.05, seed=thr + 1)
    g[rng.random(g.shape) < 0.3] = rng.integers(0, 255)
    h = as_format(g, A.FMT_GRAY8, rng, thr=thr)
    p = black_params(oracle, intensity=8, depth=(100, 100), thr=200)
    both(hip, oracle, h, lambda d: hip.blackfilter(d, p), lambda o: oracle.blackfilter(o, p))


# ---------------------------------------------------------- rotation detection
def skewed_edge(w, h, radians, fmt=A.FMT_GRAY8):  # cuda_deskew_test.c:18-33
    cx = np.float32(w) * np.float32(0.35)
    cy = np.float32(h) / np.float32(2.0)
    m = np.float32(math.tan(np.float32(radians)))
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    black = x >= cx + m * (y - cy)
    g = np.where(black, 0, 255).astype(np.uint8)
    return HostImage.from_array(g if fmt == A.FMT_GRAY8 else np.repeat(g[:, :, None], 3, 2),
                                fmt, abs_black_threshold=128)


def deskew_params(oracle, rng=5.0, step=0.1, dev=1.0, size=1500, depth=0.5,
                  edges=(True, False, True, False)):
    p = oracle.default_options().deskew_parameters
    p.deskewScanRangeRad = np.float32(np.float32(rng) * math.pi / 180.0)
    p.deskewScanStepRad = np.float32(np.float32(step) * math.pi / 180.0)
    p.deskewScanDeviationRad = np.float32(np.float32(dev) * math.pi / 180.0)
    p.deskewScanSize = size
    p.deskewScanDepth = depth
    p.scan_edges = A.Edges(*edges)
    return p


@pytest.mark.parametrize("edges", [(True, False, False, False), (True, False, True, False),
                                   (False, True, False, True), (True, True, True, True)])
def test_detect_rotation_reference_scene(hip, oracle, edges):  # cuda_deskew_test.c:86-108
    h = skewed_edge(241, 179, 2.0 * math.pi / 180.0)
    p = deskew_params(oracle, dev=10.0, size=400, edges=edges)
    mask = A.rect(0, 0, 240, 178)
    r1 = hip.detect_rotation(hip.upload(h), mask, p)
    r2 = oracle.detect_rotation(h, mask, p)
    assert np.float32(r1).tobytes() == np.float32(r2).tobytes()
    if edges[0] and not edges[2]:
        assert abs(r2) > 1e-4


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24])
@pytest.mark.parametrize("deg", [0.0, 0.6, -1.3, 3.7])
@pytest.mark.parametrize("mask", [(60, 0, 739, 599), (0, 0, 799, 599), (-20, 30, 820, 560)])
def test_detect_rotation_pages(hip, oracle, fmt, deg, mask):
    # a text block rotated by `deg` (rendered via the reference deskew itself)
    h = make_image(800, 600, fmt, seed=9, margin=90)
    if deg:
        oracle.deskew(h, A.rect(0, 0, 799, 599), float(np.float32(deg * math.pi / 180)),
                      A.INTERP_LINEAR)
    p = deskew_params(oracle, size=400)
    r1 = hip.detect_rotation(hip.upload(h), A.rect(*mask), p)
    r2 = oracle.detect_rotation(h, A.rect(*mask), p)
    assert np.float32(r1).tobytes() == np.float32(r2).tobytes()


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24])
@pytest.mark.parametrize("case", ["wide_margin", "wide_range", "scan_all"])
def test_detect_rotation_fallbacks(hip, oracle, fmt, case):
    """Lines the band path cannot finish: content > 128 steps from the mask
    edge, a 40 degree range whose band does not fit LDS, and scan size -1."""
    margin = 330 if case == "wide_margin" else 90
    h = make_image(1200, 900, fmt, seed=21, margin=margin)
    oracle.deskew(h, A.rect(0, 0, 1199, 899), float(np.float32(1.7 * math.pi / 180)),
                  A.INTERP_LINEAR)
    if case == "wide_range":
        p = deskew_params(oracle, rng=40.0, step=2.0, dev=90.0, size=1500)
    elif case == "scan_all":
        p = deskew_params(oracle, size=-1, dev=10.0)
    else:
        p = deskew_params(oracle, size=1500, dev=10.0)
    mask = A.rect(0, 0, 1199, 899)
    r1 = hip.detect_rotation(hip.upload(h), mask, p)
    r2 = oracle.detect_rotation(h, mask, p)
    assert np.float32(r1).tobytes() == np.float32(r2).tobytes()


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24])
@pytest.mark.parametrize("case", ["page", "left_edge", "wide_margin", "wide_range", "scan_all",
                                  "all_edges", "small_step"])
def test_rotation_peaks_every_line(hip, oracle, fmt, case):
    """Every (edge, angle) peak of detect_edge_rotation_peak (deskew.c:48-146),
    not only the chosen angle: the band path (segments of the float
    recurrence, u16 slice sums), the direct walks (content > 128 steps in,
    top/bottom edges, bands too wide, lines through X = 0 with many binade
    segments) against the oracle, element for element."""
    w, h, margin, deg = 1200, 900, 90, 1.7
    mask = (0, 0, w - 1, h - 1)  # left lines start at X in [0, 1): they cross X = 0
    kw = dict(size=1500, dev=10.0)
    if case == "page":
        w, h, deg, mask, kw = 800, 600, 0.6, (60, 0, 739, 599), dict(size=400)
    elif case == "wide_margin":
        margin = 330
    elif case == "wide_range":
        kw = dict(rng=40.0, step=2.0, dev=90.0, size=1500)
    elif case == "scan_all":
        kw = dict(size=-1, dev=10.0)
    elif case == "all_edges":
        kw = dict(size=700, dev=10.0, edges=(True, True, True, True))
    elif case == "small_step":
        kw = dict(rng=2.0, step=0.01, dev=10.0, size=1500)
    img = make_image(w, h, fmt, seed=21, margin=margin)
    oracle.deskew(img, A.rect(0, 0, w - 1, h - 1), float(np.float32(deg * math.pi / 180)),
                  A.INTERP_LINEAR)
    p = deskew_params(oracle, **kw)
    got = hip.detect_rotation_peaks(hip.upload(img), A.rect(*mask), p)
    exp = oracle.rotation_peaks(img, A.rect(*mask), p)
    assert got.shape == exp.shape
    # scan size -1 makes maxBlackness negative (255 * -1 * depth): every line
    # stops at once and every peak is 0 in the reference too
    assert exp.any() or case == "scan_all"
    assert np.array_equal(got, exp), np.flatnonzero(got != exp)[:20]
