"""Test helpers: deterministic synthetic pages in every pixel format, and exact
frame comparison (payload bytes; mono frames compared pixel by pixel)."""
import numpy as np

from unpaper_hip import ctypes_abi as A
from unpaper_hip.hostimage import HostImage

FORMATS = [A.FMT_GRAY8, A.FMT_RGB24, A.FMT_Y400A, A.FMT_MONOWHITE, A.FMT_MONOBLACK]
BYTE_FORMATS = [A.FMT_GRAY8, A.FMT_RGB24, A.FMT_Y400A]


def page_array(w, h, seed=0, margin=None, specks=200, color=False):
    """A scanned-page-like image: white paper, dark text blocks, salt specks,
    light-gray blotches, optional dark left band.  Returns (h, w) or (h, w, 3)."""
    rng = np.random.default_rng(seed)
    g = np.full((h, w), 255, np.uint8)
    m = margin if margin is not None else max(2, min(w, h) // 10)
    # text lines
    y = m
    while y + 12 < h - m:
        lh = int(rng.integers(4, 10))
        x = m
        while x < w - m:
            ww = int(rng.integers(3, 25))
            if x + ww >= w - m:
                break
            g[y:y + lh, x:x + ww] = rng.integers(0, 60, size=(lh, ww))
            x += ww + int(rng.integers(2, 8))
        y += lh + int(rng.integers(4, 14))
    # specks
    for _ in range(specks):
        sx, sy = int(rng.integers(0, w)), int(rng.integers(0, h))
        sw, sh = int(rng.integers(1, 3)), int(rng.integers(1, 3))
        g[sy:sy + sh, sx:sx + sw] = rng.integers(0, 120)
    # light blotches
    for _ in range(3):
        bw, bh = int(rng.integers(5, max(6, w // 5))), int(rng.integers(5, max(6, h // 5)))
        bx, by = int(rng.integers(0, max(1, w - bw))), int(rng.integers(0, max(1, h - bh)))
        blk = g[by:by + bh, bx:bx + bw]
        blk[...] = np.minimum(blk, rng.integers(180, 220, size=blk.shape))
    if not color:
        return g
    tint = rng.integers(-40, 40, size=(1, 1, 3))
    rgb = np.clip(g[:, :, None].astype(int) + tint, 0, 255).astype(np.uint8)
    # a few saturated colour patches (lightness << gray)
    for _ in range(3):
        bw, bh = int(rng.integers(5, max(6, w // 6))), int(rng.integers(5, max(6, h // 6)))
        bx, by = int(rng.integers(0, max(1, w - bw))), int(rng.integers(0, max(1, h - bh)))
        rgb[by:by + bh, bx:bx + bw] = rng.integers(0, 256, size=3).astype(np.uint8)
    return rgb


def make_image(w, h, fmt, seed=0, threshold=170, background=(255, 255, 255), **kw):
    color = fmt == A.FMT_RGB24
    arr = page_array(w, h, seed, color=color, **kw)
    if fmt == A.FMT_GRAY8:
        return HostImage.from_array(arr, fmt, abs_black_threshold=threshold, background=background)
    if fmt == A.FMT_RGB24:
        return HostImage.from_array(arr, fmt, abs_black_threshold=threshold, background=background)
    if fmt == A.FMT_Y400A:
        rng = np.random.default_rng(seed + 99)
        la = np.stack([arr, rng.integers(0, 256, size=arr.shape, dtype=np.uint8)], axis=2)
        return HostImage.from_array(la, fmt, abs_black_threshold=threshold, background=background)
    return HostImage.from_array(arr >= 128, fmt, abs_black_threshold=threshold,
                                background=background)


def frames_equal(a: HostImage, b: HostImage):
    if (a.width, a.height, a.format) != (b.width, b.height, b.format):
        return False, "geometry %r != %r" % ((a.width, a.height, a.format),
                                             (b.width, b.height, b.format))
    if a.format in (A.FMT_MONOWHITE, A.FMT_MONOBLACK):
        pa, pb = a.to_gray(), b.to_gray()
    else:
        pa, pb = a.payload(), b.payload()
    diff = np.argwhere(pa != pb)
    if len(diff):
        y, x = diff[0][:2]
        return False, "%d bytes differ, first at row %d col %d: %r vs %r" % (
            len(diff), y, x, pa[y, max(0, x - 3):x + 4], pb[y, max(0, x - 3):x + 4])
    return True, ""


def assert_same(a, b, what=""):
    ok, msg = frames_equal(a, b)
    assert ok, (what + ": " if what else "") + msg
