"""GPU parity of the ImageBackend ops: HIP result == oracle result, bit for bit,
on deterministic synthetic pages in every pixel format the op accepts.
Scenarios follow the reference's C unit tests (tests/cuda_primitives_test.c,
cuda_masks_border_test.c, cuda_deskew_test.c) plus edge cases (inverted /
outside rectangles, odd sizes, 1-pixel images)."""
import math

import numpy as np
import pytest

from unpaper_hip import ctypes_abi as A
from helpers import FORMATS, assert_same, make_image

pytestmark = pytest.mark.gpu

SIZES = [(97, 61), (256, 130), (1, 1), (33, 200)]


def run_both(hip, oracle, h, fn_hip, fn_oracle):
    d = hip.upload(h)
    ho = h.copy()
    r1 = fn_hip(d)
    r2 = fn_oracle(ho)
    out_h = d.to_host()
    return out_h, (r2 if r2 is not None and hasattr(r2, "data") else ho), r1, r2


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("size", SIZES)
def test_upload_download_roundtrip(hip, fmt, size):
    h = make_image(*size, fmt, seed=1)
    assert_same(hip.upload(h).to_host(), h)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("rect", [(5, 3, 40, 20), (-10, -10, 8, 9), (90, 50, 200, 300),
                                  (30, 40, 10, 5), (500, 500, 600, 600)])
@pytest.mark.parametrize("color", [(255, 255, 255), (0, 0, 0), (10, 200, 90)])
def test_wipe_rectangle(hip, oracle, fmt, rect, color):
    h = make_image(97, 61, fmt, seed=2)
    r, c = A.rect(*rect), A.Pixel(*color)
    d = hip.upload(h)
    hip.wipe_rectangle(d, r, c)
    oracle.wipe_rectangle(h, r, c)
    assert_same(d.to_host(), h)


@pytest.mark.parametrize("sfmt", FORMATS)
@pytest.mark.parametrize("dfmt", FORMATS)
@pytest.mark.parametrize("area,to", [((0, 0, 96, 60), (0, 0)), ((10, 5, 50, 40), (20, 7)),
                                     ((-5, -5, 30, 30), (60, 40)), ((10, 10, 60, 50), (-8, -3)),
                                     ((3, 3, 94, 58), (1, 2))])
def test_copy_rectangle(hip, oracle, sfmt, dfmt, area, to):
    s = make_image(97, 61, sfmt, seed=3)
    t = make_image(80, 55, dfmt, seed=4)
    ds, dt = hip.upload(s), hip.upload(t)
    r, p = A.rect(*area), A.Point(*to)
    hip.copy_rectangle(ds, dt, r, p)
    oracle.copy_rectangle(s, t, r, p)
    assert_same(dt.to_host(), t)


@pytest.mark.parametrize("sfmt", FORMATS)
@pytest.mark.parametrize("ssize,tsize,origin", [((60, 40), (100, 80), (0, 0)),
                                                ((100, 80), (60, 40), (0, 0)),
                                                ((60, 90), (100, 50), (10, 5)),
                                                ((50, 50), (50, 50), (25, 0))])
def test_center_image(hip, oracle, sfmt, ssize, tsize, origin):
    s = make_image(*ssize, sfmt, seed=5)
    t = make_image(120, 90, A.FMT_RGB24, seed=6, background=(0, 0, 0))
    ds, dt = hip.upload(s), hip.upload(t)
    hip.center_image(ds, dt, A.Point(*origin), A.RectangleSize(*tsize))
    oracle.center_image(s, t, A.Point(*origin), A.RectangleSize(*tsize))
    assert_same(dt.to_host(), t)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("interp", [A.INTERP_NN, A.INTERP_LINEAR, A.INTERP_CUBIC])
@pytest.mark.parametrize("size", [(150, 77), (40, 30), (97, 61), (61, 97)])
def test_stretch_and_replace(hip, oracle, fmt, interp, size):
    h = make_image(97, 61, fmt, seed=7)
    d = hip.upload(h)
    hip.stretch_and_replace(d, A.RectangleSize(*size), interp)
    ho = oracle.stretch_and_replace(h, A.RectangleSize(*size), interp)
    assert_same(d.to_host(), ho)


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24, A.FMT_MONOWHITE])
@pytest.mark.parametrize("size", [(150, 77), (40, 60), (200, 100)])
def test_resize_and_replace(hip, oracle, fmt, size):
    h = make_image(97, 61, fmt, seed=8)
    d = hip.upload(h)
    hip.resize_and_replace(d, A.RectangleSize(*size), A.INTERP_LINEAR)
    ho = oracle.resize_and_replace(h, A.RectangleSize(*size), A.INTERP_LINEAR)
    assert_same(d.to_host(), ho)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("direction", [1, -1])
@pytest.mark.parametrize("size", [(97, 61), (16, 9), (1, 5)])
def test_flip_rotate_90(hip, oracle, fmt, direction, size):
    h = make_image(*size, fmt, seed=9)
    d = hip.upload(h)
    hip.flip_rotate_90(d, direction)
    ho = oracle.flip_rotate_90(h, direction)
    assert_same(d.to_host(), ho)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("hv", [(True, False), (False, True), (True, True), (False, False)])
@pytest.mark.parametrize("size", [(97, 61), (96, 60)])
def test_mirror(hip, oracle, fmt, hv, size):
    h = make_image(*size, fmt, seed=10)
    d = hip.upload(h)
    hip.mirror(d, A.Direction(*hv))
    oracle.mirror(h, A.Direction(*hv))
    assert_same(d.to_host(), h)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("delta", [(3, -2), (-20, 15), (0, 0), (200, 0)])
def test_shift_image(hip, oracle, fmt, delta):
    h = make_image(97, 61, fmt, seed=11)
    d = hip.upload(h)
    hip.shift_image(d, A.Delta(*delta))
    ho = oracle.shift_image(h, A.Delta(*delta))
    assert_same(d.to_host(), ho)


MASK_SETS = [[(10, 10, 60, 40)], [(0, 0, 20, 20), (50, 30, 96, 60)], [(70, 50, 5, 5)],
             [(-10, -10, 200, 200)], []]


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("masks", MASK_SETS)
def test_apply_masks(hip, oracle, fmt, masks):
    h = make_image(97, 61, fmt, seed=12)
    rects = [A.rect(*m) for m in masks]
    d = hip.upload(h)
    hip.apply_masks(d, rects, A.Pixel(255, 255, 255))
    oracle.apply_masks(h, rects, A.Pixel(255, 255, 255))
    assert_same(d.to_host(), h)


@pytest.mark.parametrize("fmt", FORMATS)
def test_apply_wipes_and_border(hip, oracle, fmt):
    h = make_image(97, 61, fmt, seed=13)
    w = A.Wipes()
    areas = [(0, 0, 9, 9), (50, 50, 40, 40), (90, 55, 120, 80), (-5, 20, 3, 25)]
    w.count = len(areas)
    for i, a in enumerate(areas):
        w.areas[i] = A.rect(*a)
    d = hip.upload(h)
    hip.apply_wipes(d, w, A.Pixel(0, 0, 0))
    oracle.apply_wipes(h, w, A.Pixel(0, 0, 0))
    for b in [(2, 2, 2, 2), (0, 0, 0, 0), (10, 0, 3, 7)]:
        hip.apply_border(d, A.Border(*b), A.Pixel(255, 255, 255))
        oracle.apply_border(h, A.Border(*b), A.Pixel(255, 255, 255))
    assert_same(d.to_host(), h)


def mask_params(oracle, direction=(True, False), thr=0.1, minimum=100, size=50):
    p = oracle.default_options().mask_detection_parameters
    p.scan_direction = A.Direction(*direction)
    p.scan_threshold.horizontal = p.scan_threshold.vertical = thr
    p.minimum_width = p.minimum_height = minimum
    p.scan_size = A.RectangleSize(size, size)
    return p


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("direction", [(True, False), (False, True), (True, True)])
@pytest.mark.parametrize("thr,minimum", [(0.1, 100), (0.8, 1), (0.5, 10)])
def test_detect_masks(hip, oracle, fmt, direction, thr, minimum):
    h = make_image(400, 300, fmt, seed=14, margin=40)
    p = mask_params(oracle, direction, thr, minimum, size=20)
    p.maximum_width, p.maximum_height = 400, 300
    pts = [A.Point(200, 150), A.Point(100, 150), A.Point(300, 100)]
    d = hip.upload(h)
    n1, m1 = hip.detect_masks(d, p, pts)
    n2, m2 = oracle.detect_masks(h, p, pts)
    assert n1 == n2
    assert [m.tuple() for m in m1] == [m.tuple() for m in m2]


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("direction", [(False, True), (True, False), (True, True)])
@pytest.mark.parametrize("outside", [(0, 0, 399, 299), (0, 0, 200, 299), (200, 0, 399, 299),
                                     (10, 20, 350, 280)])
def test_detect_border(hip, oracle, fmt, direction, outside):
    h = make_image(400, 300, fmt, seed=15, margin=30)
    p = oracle.default_options().border_scan_parameters
    p.scan_direction = A.Direction(*direction)
    d = hip.upload(h)
    b1 = hip.detect_border(d, p, A.rect(*outside))
    b2 = oracle.detect_border(h, p, A.rect(*outside))
    assert b1.tuple() == b2.tuple()


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("inside,outside", [((30, 40, 300, 250), (0, 0, 399, 299)),
                                            ((0, 0, 398, 299), (0, 0, 399, 299)),
                                            ((-10, 5, 100, 320), (0, 0, 399, 299))])
@pytest.mark.parametrize("align", [(False, False, False, False), (True, True, False, False),
                                   (False, False, True, True)])
def test_align_mask(hip, oracle, fmt, inside, outside, align):
    h = make_image(400, 300, fmt, seed=16)
    p = A.MaskAlignmentParameters()
    p.alignment = A.Edges(*align)
    p.margin = A.Delta(7, 3)
    d = hip.upload(h)
    hip.align_mask(d, A.rect(*inside), A.rect(*outside), p)
    oracle.align_mask(h, A.rect(*inside), A.rect(*outside), p)
    assert_same(d.to_host(), h)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("interp", [A.INTERP_NN, A.INTERP_LINEAR, A.INTERP_CUBIC])
@pytest.mark.parametrize("deg", [2.0, -0.7, 4.9])
@pytest.mark.parametrize("mask", [(0, 0, 240, 178), (20, 15, 200, 150), (-5, 10, 250, 170)])
def test_deskew(hip, oracle, fmt, interp, deg, mask):
    h = make_image(241, 179, fmt, seed=17)
    rad = np.float32(deg * math.pi / 180.0)
    d = hip.upload(h)
    hip.deskew(d, A.rect(*mask), float(rad), interp)
    oracle.deskew(h, A.rect(*mask), float(rad), interp)
    assert_same(d.to_host(), h)


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("deg", [1.3, -12.0, 25.0, -44.0])
@pytest.mark.parametrize("mask", [(0, 0, 1029, 299), (37, 21, 990, 280)])
def test_deskew_cubic_wide(hip, oracle, fmt, deg, mask):
    # several 256-column tiles, a width that is not a multiple of 4, and angles
    # whose source windows exceed the staged height (taps read from the frame)
    h = make_image(1030, 300, fmt, seed=18)
    rad = np.float32(deg * math.pi / 180.0)
    d = hip.upload(h)
    hip.deskew(d, A.rect(*mask), float(rad), A.INTERP_CUBIC)
    oracle.deskew(h, A.rect(*mask), float(rad), A.INTERP_CUBIC)
    assert_same(d.to_host(), h)
