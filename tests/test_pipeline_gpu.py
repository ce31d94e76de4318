"""Whole-sheet parity: the HIP batch pipeline (uphip_batch_*) against the oracle's
process_sheet (oracle.c, restating sheet_process.c:134-180 and the stages of
src/core/sheet_stages.c), byte for byte on the saved output frame.

Inputs: the reference's own test sources (tests/golden/reference, with the
option sets of tests/unpaper_tests.py / cuda_pipeline_test.c that produced
the goldens) and the deterministic synthetic pages of BASELINE.md §3.
"""
import numpy as np
import pytest

from helpers import assert_same, page_array
from unpaper_hip import ctypes_abi as A
from unpaper_hip.hostimage import HostImage
from unpaper_hip.pipeline import Batch, DeviceBuffer, synth_page_host

pytestmark = pytest.mark.gpu


def oracle_sheet(oracle, opts, pages):
    sheet, fmt, rep = oracle.process_sheet(opts, pages)
    return oracle.convert_for_save(sheet, fmt), rep


def gpu_sheets(opts, sheets, bg=None):
    """sheets: list of page lists (all pages the same geometry)."""
    p0 = sheets[0][0]
    b = Batch(opts, len(sheets), p0.width, p0.height, p0.format)
    try:
        for s, pages in enumerate(sheets):
            for j, p in enumerate(pages):
                b.set_input(s, j, p)
        b.run(len(sheets))
        b.wait()
        outs = [b.output(s) for s in range(len(sheets))]
        reps = [b.report(s) for s in range(len(sheets))]
        return outs, reps
    finally:
        b.close()


def check(oracle, opts, sheets, what=""):
    outs, reps = gpu_sheets(opts, sheets)
    for s, pages in enumerate(sheets):
        exp, erep = oracle_sheet(oracle, opts, pages)
        assert_same(outs[s], exp, "%s sheet %d" % (what, s))
        assert reps[s].mask_count == erep.mask_count
        for i in range(min(erep.mask_count, A.MAX_PAGES)):
            assert np.float32(reps[s].rotation[i]).tobytes() == \
                np.float32(erep.rotation[i]).tobytes(), "rotation %d" % i
    return outs


def synth(w, h, page, fmt=A.FMT_GRAY8, threshold=170):
    g = synth_page_host(w, h, page)
    if fmt == A.FMT_GRAY8:
        return HostImage.from_array(g, fmt, abs_black_threshold=threshold)
    rng = np.random.default_rng(page)
    tint = rng.integers(-30, 30, size=(1, 1, 3))
    rgb = np.clip(g[:, :, None].astype(int) + tint, 0, 255).astype(np.uint8)
    return HostImage.from_array(rgb, A.FMT_RGB24, abs_black_threshold=threshold)


SMALL = (620, 877)   # A4 at 75 dpi: full pipeline, oracle in well under a second


# ---------------------------------------------------------------------------
# synthetic pages
# ---------------------------------------------------------------------------
def test_synth_device_matches_host(hip):
    w, h, n = 333, 250, 5
    pitch = 512
    buf = DeviceBuffer(pitch * h * n)
    L = buf.lib
    assert L.uphip_synth_pages(buf.ptr, pitch, pitch * h, w, h, 7, n) == 0
    host = np.empty((n, h, pitch), np.uint8)
    assert L.uphip_memcpy_dtoh(host.ctypes.data, buf.ptr, host.nbytes) == 0
    for i in range(n):
        assert np.array_equal(host[i, :, :w], synth_page_host(w, h, 7 + i)), i
    buf.close()


def test_default_gray_batch(hip, oracle):
    opts = oracle.default_options()
    sheets = [[synth(*SMALL, p)] for p in range(6)]   # page 3: dark band (blackfilter)
    check(oracle, opts, sheets, "default")


def test_default_rgb_batch(hip, oracle):
    opts = oracle.default_options()
    sheets = [[synth(*SMALL, p, A.FMT_RGB24)] for p in (1, 3, 4)]
    check(oracle, opts, sheets, "rgb")


def test_default_a4_pages(hip, oracle):
    opts = oracle.default_options()
    sheets = [[synth(2480, 3508, p)] for p in (0, 3)]
    check(oracle, opts, sheets, "a4")


def test_run_device_matches_run(hip, oracle):
    opts = oracle.default_options()
    w, h, n = SMALL[0], SMALL[1], 4
    pitch = (w + 255) // 256 * 256
    buf = DeviceBuffer(pitch * h * n)
    assert buf.lib.uphip_synth_pages(buf.ptr, pitch, pitch * h, w, h, 20, n) == 0
    b = Batch(opts, n, w, h, A.FMT_GRAY8)
    b.run_device(n, buf.ptr, pitch, pitch * h)
    b.wait()
    dev = [b.output(s) for s in range(n)]
    # second run on fewer sheets reuses the batch
    b.run_device(2, buf.ptr, pitch, pitch * h)
    b.wait()
    again = [b.output(s) for s in range(2)]
    b.close()
    for s in range(n):
        exp, _ = oracle_sheet(oracle, opts, [synth(w, h, 20 + s)])
        assert_same(dev[s], exp, "device input sheet %d" % s)
    for s in range(2):
        assert_same(again[s], dev[s], "rerun sheet %d" % s)


# ---------------------------------------------------------------------------
# option coverage (sheet_stages.c stages one by one)
# ---------------------------------------------------------------------------
STAGE_BITS = [A.NO_BLACKFILTER, A.NO_NOISEFILTER, A.NO_BLURFILTER, A.NO_GRAYFILTER,
              A.NO_MASK_SCAN, A.NO_MASK_CENTER, A.NO_DESKEW, A.NO_WIPE, A.NO_BORDER,
              A.NO_BORDER_SCAN, A.NO_BORDER_ALIGN]


@pytest.mark.parametrize("bit", STAGE_BITS)
def test_stage_disabled(hip, oracle, bit):
    opts = oracle.default_options()
    opts.disable = bit
    check(oracle, opts, [[synth(*SMALL, 3)], [synth(*SMALL, 5)]], "disable %#x" % bit)


@pytest.mark.parametrize("only", STAGE_BITS)
def test_stage_only(hip, oracle, only):
    opts = oracle.default_options()
    opts.disable = A.NO_PROCESSING & ~only
    check(oracle, opts, [[synth(*SMALL, 2)], [synth(*SMALL, 3)]], "only %#x" % only)


def test_no_processing(hip, oracle):
    opts = oracle.default_options()
    opts.disable = A.NO_PROCESSING
    check(oracle, opts, [[synth(*SMALL, 1)]], "-n")


@pytest.mark.parametrize("interp", [A.INTERP_NN, A.INTERP_LINEAR, A.INTERP_CUBIC])
def test_deskew_interpolation(hip, oracle, interp):
    opts = oracle.default_options()
    opts.interpolate_type = interp
    check(oracle, opts, [[synth(*SMALL, p)] for p in (0, 1, 2)], "interp %d" % interp)


@pytest.mark.parametrize("edges", [(True, True, True, True), (False, True, False, True),
                                   (True, False, False, False)])
def test_deskew_edges(hip, oracle, edges):
    opts = oracle.default_options()
    opts.deskew_parameters.scan_edges = A.Edges(*edges)
    check(oracle, opts, [[synth(*SMALL, p)] for p in (0, 1)], "edges %r" % (edges,))


def frame_page(w, h, deg, seed=1):
    """White page with a 12-px dark rectangular frame (60 % of the page)
    rotated by `deg` about the centre: all four mask edges see the same
    slope, so every edge set agrees within the deviation and the combined
    rotation is non-zero (the synthetic text pages' top/bottom edges do not
    agree with the left/right ones)."""
    import math
    rng = np.random.default_rng(seed)
    bw, bh = int(w * 0.6), int(h * 0.6)
    t = math.radians(deg)
    yy, xx = np.mgrid[0:h, 0:w]
    dx, dy = xx - w / 2 + 0.5, yy - h / 2 + 0.5
    u = math.cos(t) * dx + math.sin(t) * dy
    v = -math.sin(t) * dx + math.cos(t) * dy
    frame = (np.abs(u) < bw / 2) & (np.abs(v) < bh / 2) & \
        ~((np.abs(u) < bw / 2 - 12) & (np.abs(v) < bh / 2 - 12))
    g = np.where(frame, rng.integers(0, 40, size=(h, w)), 255).astype(np.uint8)
    return HostImage.from_array(g, A.FMT_GRAY8, abs_black_threshold=170)


@pytest.mark.parametrize("edges", [(True, True, True, False), (True, True, True, True),
                                   (False, True, False, True)])
@pytest.mark.parametrize("interp", [A.INTERP_CUBIC, A.INTERP_LINEAR])
def test_deskew_multi_edge_nonzero(hip, oracle, edges, interp):
    """the batch path's rotation select with 3 and 4 edges
    (device glibc sinf/cosf/powf, libm_glibc.h) and the top/bottom edges
    (deskew.c:96-97 sideOffset), with NON-ZERO oracle rotations, whole
    sheets against the oracle."""
    opts = oracle.default_options()
    opts.interpolate_type = interp
    opts.deskew_parameters.scan_edges = A.Edges(*edges)
    degs = (1.3, 0.65, -2.2, 3.7)
    sheets = [[frame_page(*SMALL, d)] for d in degs]
    check(oracle, opts, sheets, "edges %r" % (edges,))
    rots = [float(oracle_sheet(oracle, opts, p)[1].rotation[0]) for p in sheets]
    assert sum(r != 0.0 for r in rots) >= 2, rots
    if sum(edges) > 2:
        # an average of disagreeing edges: not itself an angle of the scan table
        step = np.float32(np.radians(0.1))
        assert any(r != 0.0 and abs(r / step - round(r / step)) > 1e-3 for r in rots), rots


@pytest.mark.parametrize("rot", [90, -90])
def test_pre_post_rotate(hip, oracle, rot):
    opts = oracle.default_options()
    opts.pre_rotate = rot
    opts.post_rotate = -rot
    check(oracle, opts, [[synth(*SMALL, 1)]], "rotate %d" % rot)


def test_mirror_shift(hip, oracle):
    opts = oracle.default_options()
    opts.pre_mirror = A.Direction(True, False)
    opts.post_mirror = A.Direction(False, True)
    opts.pre_shift = A.Delta(17, -9)
    opts.post_shift = A.Delta(-5, 23)
    check(oracle, opts, [[synth(*SMALL, 4)]], "mirror/shift")


@pytest.mark.parametrize("interp", [A.INTERP_NN, A.INTERP_LINEAR, A.INTERP_CUBIC])
def test_sizes(hip, oracle, interp):
    opts = oracle.default_options()
    opts.interpolate_type = interp
    opts.stretch_size = A.RectangleSize(700, 900)
    opts.pre_zoom_factor = 0.8
    opts.page_size = A.RectangleSize(600, 800)
    opts.post_stretch_size = A.RectangleSize(500, 700)
    opts.post_page_size = A.RectangleSize(520, 640)
    check(oracle, opts, [[synth(*SMALL, 2)]], "sizes %d" % interp)


def test_sheet_size_and_background(hip, oracle):
    opts = oracle.default_options()
    opts.sheet_size = A.RectangleSize(700, 1000)
    opts.sheet_background = A.pixel(0)
    check(oracle, opts, [[synth(*SMALL, 1)]], "sheet size")


def test_wipes_borders_masks(hip, oracle):
    opts = oracle.default_options()
    opts.pre_wipes.count = 2
    opts.pre_wipes.areas[0] = A.rect(0, 0, 49, 39)
    opts.pre_wipes.areas[1] = A.rect(500, 800, 700, 900)
    opts.wipes.count = 1
    opts.wipes.areas[0] = A.rect(300, 10, 330, 860)
    opts.post_wipes.count = 1
    opts.post_wipes.areas[0] = A.rect(-5, 600, 100, 620)
    opts.pre_border = A.Border(3, 4, 5, 6)
    opts.border = A.Border(10, 0, 0, 12)
    opts.post_border = A.Border(0, 7, 7, 0)
    opts.pre_mask_count = 1
    opts.pre_masks[0] = A.rect(20, 30, 580, 840)
    check(oracle, opts, [[synth(*SMALL, 0)], [synth(*SMALL, 3)]], "wipes")


def test_points_and_mask_params(hip, oracle):
    opts = oracle.default_options()
    opts.point_count = 2
    opts.points[0] = A.Point(200, 300)
    opts.points[1] = A.Point(450, 600)
    mp = opts.mask_detection_parameters
    mp.scan_direction = A.Direction(True, True)
    mp.scan_threshold.horizontal = 0.2
    mp.scan_threshold.vertical = 0.2
    mp.minimum_width = 50
    mp.minimum_height = 50
    opts.mask_alignment_parameters.alignment = A.Edges(True, True, False, False)
    opts.mask_alignment_parameters.margin = A.Delta(12, 8)
    check(oracle, opts, [[synth(*SMALL, 1)], [synth(*SMALL, 2)]], "points")


def test_border_scan_align(hip, oracle):
    opts = oracle.default_options()
    bp = opts.border_scan_parameters
    bp.scan_direction = A.Direction(True, True)
    bp.scan_size = A.RectangleSize(10, 10)
    bp.scan_step = A.Delta(3, 3)
    bp.scan_threshold.horizontal = 2
    bp.scan_threshold.vertical = 2
    opts.mask_alignment_parameters.alignment = A.Edges(False, True, False, False)
    check(oracle, opts, [[synth(*SMALL, 0)], [synth(*SMALL, 5)]], "border")


def test_filter_parameters(hip, oracle):
    opts = oracle.default_options()
    opts.noisefilter_intensity = 2
    opts.blurfilter_parameters.scan_size = A.RectangleSize(60, 60)
    opts.blurfilter_parameters.scan_step = A.Delta(30, 30)
    opts.blurfilter_parameters.intensity = 0.05
    opts.grayfilter_parameters.scan_size = A.RectangleSize(40, 40)
    opts.grayfilter_parameters.scan_step = A.Delta(20, 20)
    opts.grayfilter_parameters.abs_threshold = 100
    bf = opts.blackfilter_parameters
    bf.scan_size = A.RectangleSize(30, 30)
    bf.scan_step = A.Delta(10, 10)
    bf.abs_threshold = 230
    bf.intensity = 10
    check(oracle, opts, [[synth(*SMALL, 3)], [synth(*SMALL, 4)]], "filters")


def speckled(w, h, page, per_rect, seed):
    """Synthetic page `page` over its top half; below, blank paper holding
    isolated black specks (the noisefilter clears them) and specks at the
    white threshold 229 (dark for the blurfilter only) at `per_rect` per
    100x100 blurfilter block, near the default wipe threshold of 100, plus a
    solid bar on the left edge (the blackfilter paints it): the blurfilter's
    block counts hold only if its bit-plane lost what the other two cleared."""
    g = synth_page_host(w, h, page).copy()
    rng = np.random.default_rng(seed)
    y0 = h // 2
    g[y0:] = 255
    area = (h - y0) * w // 10000
    for val, n in ((0, 150 * area), (229, per_rect * area)):
        ys, xs = rng.integers(y0, h, n), rng.integers(0, w, n)
        g[ys, xs] = val
    g[y0:, 0:60] = 0
    return HostImage.from_array(g, A.FMT_GRAY8, abs_black_threshold=170)


@pytest.mark.parametrize("white", [229, 255])
def test_blur_counts_after_noise_and_black_clears(hip, oracle, white):
    # the fused GRAY8 decode's blurfilter bit-plane (pixel <= white), kept by
    # the blackfilter's paint and the noisefilter's clears (off at white 255:
    # a cleared pixel would still count); the grayfilter, which would wipe
    # the blocks anyway, is off
    opts = oracle.default_options()
    opts.abs_white_threshold = white
    opts.disable |= A.NO_GRAYFILTER
    sheets = [[speckled(*SMALL, p, k, 10 * p + k)] for p, k in ((3, 40), (0, 70), (3, 90), (5, 110))]
    check(oracle, opts, sheets, "blur bits")


def test_noisefilter_sequential_intensity(hip, oracle):
    opts = oracle.default_options()
    opts.noisefilter_intensity = 6
    check(oracle, opts, [[synth(320, 440, 3)]], "noise 6")


def test_threshold_options(hip, oracle):
    opts = oracle.default_options()
    opts.abs_black_threshold = 120
    opts.abs_white_threshold = 200
    check(oracle, opts, [[synth(*SMALL, 1, threshold=120)], [synth(*SMALL, 3, threshold=120)]],
          "thresholds")


@pytest.mark.parametrize("fmt", [A.FMT_GRAY8, A.FMT_RGB24, A.FMT_MONOWHITE])
def test_output_pixel_format(hip, oracle, fmt):
    opts = oracle.default_options()
    opts.output_pixel_format = fmt
    check(oracle, opts, [[synth(*SMALL, 2, A.FMT_RGB24)]], "outfmt %d" % fmt)


def test_colour_mask_forces_rgb_plane(hip, oracle):
    opts = oracle.default_options()
    opts.mask_color = A.Pixel(255, 0, 0)
    opts.border = A.Border(20, 20, 20, 20)
    opts.output_pixel_format = A.FMT_RGB24
    check(oracle, opts, [[synth(*SMALL, 1)]], "red mask")


def test_mono_and_y400a_inputs(hip, oracle):
    opts = oracle.default_options()
    g = synth_page_host(*SMALL, 6)
    mono = HostImage.from_array(g >= 128, A.FMT_MONOWHITE)
    check(oracle, opts, [[mono]], "mono")
    la = np.stack([g, np.full_like(g, 200)], axis=2)
    check(oracle, opts, [[HostImage.from_array(la, A.FMT_Y400A)]], "y400a")


# ---------------------------------------------------------------------------
# layouts
# ---------------------------------------------------------------------------
def test_double_layout_two_outputs(hip, oracle):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.output_count = 2
    wide = [np.concatenate([synth_page_host(*SMALL, p), synth_page_host(*SMALL, p + 1)], axis=1)
            for p in (0, 2)]
    sheets = [[HostImage.from_array(a, A.FMT_GRAY8)] for a in wide]
    check(oracle, opts, sheets, "double")


def test_two_inputs_double_layout(hip, oracle):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.input_count = 2
    sheets = [[synth(*SMALL, 0), synth(*SMALL, 1)], [synth(*SMALL, 4), synth(*SMALL, 3)]]
    check(oracle, opts, sheets, "two inputs")


def test_middle_wipe(hip, oracle):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.middle_wipe[0] = 15
    opts.middle_wipe[1] = 25
    wide = np.concatenate([synth_page_host(*SMALL, 5), synth_page_host(*SMALL, 6)], axis=1)
    check(oracle, opts, [[HostImage.from_array(wide, A.FMT_GRAY8)]], "middle wipe")


def test_layout_none(hip, oracle):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_NONE
    check(oracle, opts, [[synth(*SMALL, 2)]], "layout none")


# ---------------------------------------------------------------------------
# the reference's own integration sources and option sets
# (tests/unpaper_tests.py: A1, C1, C2, E1, F)
# ---------------------------------------------------------------------------
def load(ref_path, name, opts):
    return HostImage.load(ref_path(name), abs_black_threshold=opts.abs_black_threshold,
                          background=(opts.sheet_background.r,) * 3)


def test_golden_A1(hip, oracle, ref_path):
    opts = oracle.default_options()
    check(oracle, opts, [[load(ref_path, "imgsrc001.png", opts)]], "A1")


@pytest.mark.parametrize("case", ["C1", "C2"])
def test_golden_C_pbm(hip, oracle, ref_path, case):
    opts = oracle.default_options()
    opts.disable = A.NO_PROCESSING
    opts.sheet_size = A.RectangleSize(2480, 3508)
    if case == "C1":
        opts.sheet_background = A.pixel(0)
    else:
        opts.pre_shift = A.Delta(-591, 1063)
    check(oracle, opts, [[load(ref_path, "imgsrc002.png", opts)]], case)


def test_golden_C1_ppm(hip, oracle, ref_path):
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
    check(oracle, opts, [[load(ref_path, "imgsrc006.png", opts)]], "C1 ppm")


def test_golden_E1(hip, oracle, ref_path):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.output_count = 2
    for name in ("imgsrcE001.png", "imgsrcE002.png", "imgsrcE003.png"):
        check(oracle, opts, [[load(ref_path, name, opts)]], name)


def test_golden_F(hip, oracle, ref_path):
    opts = oracle.default_options()
    opts.layout = A.LAYOUT_DOUBLE
    opts.input_count = 2
    pages = [load(ref_path, "imgsrcE001.png", opts), load(ref_path, "imgsrcE002.png", opts)]
    check(oracle, opts, [pages], "F")


def test_reference_sources_batch(hip, oracle, ref_path):
    """Sources of identical geometry batched into one launch sequence."""
    opts = oracle.default_options()
    srcs = [load(ref_path, n, opts) for n in ("imgsrc003.png", "imgsrc004.png", "imgsrc005.png")]
    groups = {}
    for s in srcs:
        groups.setdefault((s.width, s.height, s.format), []).append([s])
    for sheets in groups.values():
        check(oracle, opts, sheets, "sources")


def centered_page(w, h):
    """A text-like block exactly in the middle of the sheet (the center
    stage's move is then the identity, MoveArgs.active = 0), plus a dark
    speckle row near the top for the border scan."""
    g = np.full((h, w), 255, np.uint8)
    bw, bh = w // 2, h // 2
    x0, y0 = (w - bw) // 2, (h - bh) // 2
    rng = np.random.default_rng(11)
    blk = rng.integers(0, 256, size=(bh, bw))
    g[y0:y0 + bh, x0:x0 + bw] = np.where(blk < 90, 20, 255).astype(np.uint8)
    g[y0 - 30:y0 - 26, x0:x0 + bw // 3] = 30
    return HostImage.from_array(g, A.FMT_GRAY8, abs_black_threshold=170)


def test_center_move_border_counts(hip, oracle):
    """Center moves that are the identity (MoveArgs.active = 0, the plane is
    not flipped) next to real moves in one batch, followed by the border
    scan, with and without a wipe in between, against the oracle."""
    opts = oracle.default_options()
    sheets = [[centered_page(*SMALL)], [synth(*SMALL, 0)], [centered_page(*SMALL)],
              [synth(*SMALL, 3)]]
    check(oracle, opts, sheets, "center + border")
    opts.wipes.count = 1
    opts.wipes.areas[0] = A.rect(5, 5, 40, 60)
    check(oracle, opts, sheets, "center + wipe + border")


# ---------------------------------------------------------------------------
# the two-launch GRAY8 bicubic rotation (kernels_blit.hip launch_rotate_mask)
# ---------------------------------------------------------------------------
def skewed_page(w, h, deg, seed):
    """White page, a block of 3x3-cell text lines rotated by `deg` degrees
    about the centre (nearest neighbour), so rotation detection finds about
    `deg` and the deskew rotates by it."""
    import math
    rng = np.random.default_rng(seed)
    cw, ch = int(w * 0.7), int(h * 0.7)
    g = np.full((ch, cw), 255, np.uint8)
    for y in range(0, ch - 10, 20):
        cells = rng.random((3, cw // 3)) < 0.4
        vals = rng.integers(0, 41, size=cells.shape)
        blk = np.where(cells, vals, 255).astype(np.uint8)
        g[y:y + 9, :cells.shape[1] * 3] = np.repeat(np.repeat(blk, 3, 0), 3, 1)
    out = np.full((h, w), 255, np.uint8)
    t = math.radians(deg)
    yy, xx = np.mgrid[0:h, 0:w]
    dx, dy = xx - w / 2, yy - h / 2
    u = (math.cos(t) * dx + math.sin(t) * dy + cw / 2).astype(np.int64)
    v = (-math.sin(t) * dx + math.cos(t) * dy + ch / 2).astype(np.int64)
    ok = (u >= 0) & (u < cw) & (v >= 0) & (v < ch)
    out[ok] = g[v[ok], u[ok]]
    return out


def test_rotate_window_classes_batch(hip, oracle):
    """one batch of 70 sheets (more than the persistent launch's
    64-sheet ballot) whose angles fall on both sides of the small-window
    bound (59 window rows: |angle| <= ~2.7 deg at 128-column tiles), mixed
    with blank sheets (no rotation) -- both launches take sheets, the
    large-window one through its ballot/ffs sheet walk over two 64-sheet
    groups.  Every sheet and detected angle against the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    opts = oracle.default_options()
    w, h = 400, 560
    degs = [1.0, 2.6, 2.8, 4.9, -4.9, -2.75, None, 2.65, -1.2, 3.9]
    sheets = []
    for i in range(70):
        d = degs[i % len(degs)]
        a = np.full((h, w), 255, np.uint8) if d is None else skewed_page(w, h, d, i)
        sheets.append([HostImage.from_array(a, A.FMT_GRAY8)])
    outs, reps = gpu_sheets(opts, sheets)
    with ThreadPoolExecutor(8) as ex:
        exps = list(ex.map(lambda p: oracle_sheet(oracle, opts, p), sheets))
    large = small = 0
    for s, (exp, erep) in enumerate(exps):
        assert_same(outs[s], exp, "rotate class sheet %d" % s)
        assert np.float32(reps[s].rotation[0]).tobytes() == \
            np.float32(erep.rotation[0]).tobytes(), "rotation of sheet %d" % s
        r = abs(float(erep.rotation[0]))
        if r:
            need = 48 + int(np.ceil(127 * np.sin(np.float32(r)))) + 5
            large += need > 59
            small += need <= 59
    assert large >= 20 and small >= 20, (large, small)


def _blank_band(w, h, page, top, bottom):
    """Synthetic page `page` with rows [0, top) and [h - bottom, h) made white:
    the border scan from that edge finds its first dark band only past them."""
    g = synth_page_host(w, h, page).copy()
    g[:top] = 255
    if bottom:
        g[-bottom:] = 255
    return HostImage.from_array(g, A.FMT_GRAY8, abs_black_threshold=170)


@pytest.mark.parametrize("margins", [(0, 0), (400, 0), (0, 450), (420, 430), (700, 10)])
@pytest.mark.parametrize("align", ["center", "top", "bottom_right"])
def test_chained_center_border_align(hip, oracle, margins, align):
    """The centring move, the border scan and the masked align move chained
    (pipeline.hip chain_center_align, kernels_blit.hip k_move_chain_g16):
    the scan first counts only the rows within 320 of each edge; pages whose
    margin is wider (the top, the bottom or both blanked past 320 rows) make
    it count the middle rows and scan again.  Whole sheets against the
    oracle, which centres, scans and aligns in three steps."""
    opts = oracle.default_options()
    if align == "top":
        opts.mask_alignment_parameters.alignment = A.Edges(False, True, False, False)
    elif align == "bottom_right":
        opts.mask_alignment_parameters.alignment = A.Edges(False, False, True, True)
        opts.mask_alignment_parameters.margin = A.Delta(7, 11)
    w, h = 1240, 1754  # A4 at 150 dpi: > 2 x 320 + 64 rows
    sheets = [[_blank_band(w, h, p, *margins)] for p in (2, 7)]
    check(oracle, opts, sheets, "margins %r align %s" % (margins, align))
