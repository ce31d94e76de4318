"""Pins the oracle to the reference's own golden images (CPU only).

The option sets follow tests/unpaper_tests.py in the reference (test ids A1,
C1 pbm/ppm, C2, E1, F); the fixtures under tests/golden/reference are the
reference's source and golden images re-encoded losslessly as PNG (see
tests/golden/make_fixtures.py).  The reference compares binarized images and
accepts small ratios; the bounds below are what this oracle reaches (A1 equals
the reference's own CPU build's 1.79e-5 recorded in SURVEY.md §8c).
"""
import numpy as np
import pytest
from PIL import Image

from unpaper_hip import ctypes_abi as A
from unpaper_hip.hostimage import HostImage, binarized_diff_ratio


def load(ref_path, name, opts):
    return HostImage.load(ref_path(name), abs_black_threshold=opts.abs_black_threshold,
                          background=(opts.sheet_background.r,) * 3)


def golden(ref_path, name):
    with Image.open(ref_path(name)) as im:
        return np.array(im.convert("L"))


def gray(h):
    return np.array(h.to_pil().convert("L"))


def outputs(oracle, opts, pages):
    sheet, fmt, rep = oracle.process_sheet(opts, pages)
    if opts.output_count == 1:
        return [oracle.convert_for_save(sheet, fmt)], rep
    w = sheet.width // opts.output_count
    outs = []
    for j in range(opts.output_count):
        page = HostImage(w, sheet.height, sheet.format, background=sheet.background,
                         abs_black_threshold=sheet.abs_black_threshold)
        oracle.copy_rectangle(sheet, page, A.rect(w * j, 0, w * j + w, sheet.height),
                              A.Point(0, 0))
        outs.append(oracle.convert_for_save(page, fmt))
    return outs, rep


def test_golden_A1(oracle, ref_path):
    opts = oracle.default_options()
    (out,), rep = outputs(oracle, opts, [load(ref_path, "imgsrc001.png", opts)])
    assert out.format == A.FMT_MONOWHITE
    assert binarized_diff_ratio(golden(ref_path, "goldenA1_pbm.png"), gray(out)) <= 2e-5


@pytest.mark.parametrize("case", ["C1", "C2"])
def test_golden_C_pbm(oracle, ref_path, case):
    opts = oracle.default_options()
    opts.disable = A.NO_PROCESSING
    opts.sheet_size = A.RectangleSize(2480, 3508)
    if case == "C1":
        opts.sheet_background = A.pixel(0)
    else:
        opts.pre_shift = A.Delta(-591, 1063)
    (out,), _ = outputs(oracle, opts, [load(ref_path, "imgsrc002.png", opts)])
    assert binarized_diff_ratio(golden(ref_path, "golden%s_pbm.png" % case), gray(out)) == 0


def test_golden_C1_ppm(oracle, ref_path):
    opts = oracle.default_options()
    opts.disable = (A.NO_DESKEW | A.NO_BLACKFILTER | A.NO_NOISEFILTER | A.NO_BLURFILTER |
                    A.NO_GRAYFILTER | A.NO_MASK_CENTER)
    mp = opts.mask_detection_parameters
    mp.scan_direction = A.Direction(True, True)
    mp.scan_threshold.horizontal = 0.8
    mp.scan_threshold.vertical = 0.8
    mp.minimum_width = 1
    mp.minimum_height = 1
    opts.border_scan_parameters.scan_direction = A.Direction(True, True)
    opts.pre_wipes.count = 1
    opts.pre_wipes.areas[0] = A.rect(0, 0, 9, 9)
    opts.pre_border = A.Border(2, 2, 2, 2)
    (out,), _ = outputs(oracle, opts, [load(ref_path, "imgsrc006.png", opts)])
    with Image.open(ref_path("goldenC1_ppm.png")) as im:
        g = np.array(im.convert("RGB"))
    assert np.array_equal(out.to_rgb(), g)


def test_golden_E1(oracle, ref_path):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.output_count = 2
    k = 1
    for name in ("imgsrcE001.png", "imgsrcE002.png", "imgsrcE003.png"):
        outs, _ = outputs(oracle, opts, [load(ref_path, name, opts)])
        for out in outs:
            r = binarized_diff_ratio(golden(ref_path, "goldenE1-%02d_pbm.png" % k), gray(out))
            assert r <= 1e-5, (k, r)
            k += 1


def test_golden_F(oracle, ref_path):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.input_count = 2
    pages = [load(ref_path, "imgsrcE001.png", opts), load(ref_path, "imgsrcE002.png", opts)]
    (out,), _ = outputs(oracle, opts, pages)
    assert binarized_diff_ratio(golden(ref_path, "goldenF_pbm.png"), gray(out)) == 0
