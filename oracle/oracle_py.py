"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
import ctypes as C
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG_PY = os.path.join(os.path.dirname(_HERE), "unpaper-gpu_amd", "python")
if _PKG_PY not in sys.path:
    sys.path.insert(0, _PKG_PY)

from unpaper_hip import ctypes_abi as A  # noqa: E402
from unpaper_hip.hostimage import HostImage  # noqa: E402

LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")


class OImage(C.Structure):
    _fields_ = [
        ("data", C.POINTER(C.c_uint8)),
        ("linesize", C.c_int64),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("format", C.c_int32),
        ("background", A.Pixel),
        ("abs_black_threshold", C.c_uint8),
    ]


class OStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "flood_fill_calls", "flood_fill_matches", "flood_fill_max_depth",
        "noise_clusters", "blackfilter_fills")]


def _build():
    import subprocess
    subprocess.check_call(["make", "-s", "oracle"], cwd=os.path.dirname(_HERE))


class Oracle:
    def __init__(self, path=LIB_PATH, build=True):
        if not os.path.exists(path) and build:
            _build()
        self.lib = L = C.CDLL(path)
        img, pimg = OImage, C.POINTER(OImage)
        sig = {
            "o_create_image": (img, [A.RectangleSize, C.c_int32, C.c_bool, A.Pixel, C.c_uint8]),
            "o_free_image": (None, [pimg]),
            "o_wipe_rectangle": (None, [img, A.Rectangle, A.Pixel]),
            "o_copy_rectangle": (None, [img, img, A.Rectangle, A.Point]),
            "o_center_image": (None, [img, img, A.Point, A.RectangleSize]),
            "o_stretch_and_replace": (None, [pimg, A.RectangleSize, C.c_int32]),
            "o_resize_and_replace": (None, [pimg, A.RectangleSize, C.c_int32]),
            "o_flip_rotate_90": (None, [pimg, C.c_int32]),
            "o_mirror": (None, [img, A.Direction]),
            "o_shift_image": (None, [pimg, A.Delta]),
            "o_apply_masks": (None, [img, C.POINTER(A.Rectangle), C.c_size_t, A.Pixel]),
            "o_apply_wipes": (None, [img, C.POINTER(A.Wipes), A.Pixel]),
            "o_apply_border": (None, [img, A.Border, A.Pixel]),
            "o_detect_masks": (C.c_size_t, [img, C.POINTER(A.MaskDetectionParameters),
                                            C.POINTER(A.Point), C.c_size_t,
                                            C.POINTER(A.Rectangle)]),
            "o_align_mask": (None, [img, A.Rectangle, A.Rectangle, A.MaskAlignmentParameters]),
            "o_detect_border": (A.Border, [img, A.BorderScanParameters, A.Rectangle]),
            "o_blackfilter": (None, [img, C.POINTER(A.BlackfilterParameters)]),
            "o_blurfilter": (None, [img, A.BlurfilterParameters, C.c_uint8]),
            "o_noisefilter": (None, [img, C.c_uint64, C.c_uint8]),
            "o_grayfilter": (None, [img, A.GrayfilterParameters]),
            "o_detect_rotation": (C.c_float, [img, A.Rectangle, C.POINTER(A.DeskewParameters)]),
            "o_rotation_peaks": (C.c_int, [img, A.Rectangle, C.POINTER(A.DeskewParameters),
                                           C.c_void_p, C.c_int]),
            "o_deskew": (None, [img, A.Rectangle, C.c_float, C.c_int32]),
            "o_center_mask": (None, [img, A.Point, A.Rectangle]),
            "o_process_sheet": (C.c_int, [C.POINTER(A.Options), C.POINTER(OImage), pimg,
                                          C.POINTER(C.c_int32), C.POINTER(A.SheetReport)]),
            "o_convert_for_save": (img, [img, C.c_int32]),
            "o_options_init": (None, [C.POINTER(A.Options)]),
            "o_stats_get": (None, [C.POINTER(OStats)]),
            "o_stats_reset": (None, []),
            "oracle_abi_sizeof": (C.c_size_t, [C.c_char_p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args

    # -- conversions -------------------------------------------------------
    @staticmethod
    def wrap(h: HostImage) -> OImage:
        """OImage view over a HostImage buffer (no copy; ops mutate it)."""
        o = OImage()
        o.data = h.data.ctypes.data_as(C.POINTER(C.c_uint8))
        o.linesize = h.linesize
        o.width, o.height, o.format = h.width, h.height, h.format
        o.background = A.Pixel(*h.background)
        o.abs_black_threshold = h.abs_black_threshold
        return o

    def adopt(self, o: OImage) -> HostImage:
        """Copy a C-allocated OImage into a HostImage and free it."""
        n = o.linesize * o.height
        buf = np.ctypeslib.as_array(o.data, shape=(max(n, 1),))[:n].copy()
        h = HostImage(o.width, o.height, o.format, buf.reshape(o.height, o.linesize),
                      (o.background.r, o.background.g, o.background.b),
                      o.abs_black_threshold)
        self.lib.o_free_image(C.byref(o))
        return h

    def _replace(self, fn, h: HostImage, *args) -> HostImage:
        """Run an op that replaces the frame (Image*): work on a C copy."""
        o = self.lib.o_create_image(A.RectangleSize(h.width, h.height), h.format, False,
                                    A.Pixel(*h.background), h.abs_black_threshold)
        dst = np.ctypeslib.as_array(o.data, shape=(o.linesize * o.height,))
        dst.reshape(o.height, o.linesize)[:, :h.linesize] = h.data[:, :o.linesize]
        fn(C.byref(o), *args)
        return self.adopt(o)

    # -- options -----------------------------------------------------------
    def default_options(self):
        o = A.Options()
        self.lib.o_options_init(C.byref(o))
        return o

    # -- ops (in place on HostImage unless they replace the frame) ----------
    def wipe_rectangle(self, h, r, color):
        self.lib.o_wipe_rectangle(self.wrap(h), r, color)

    def copy_rectangle(self, src, dst, r, pt):
        self.lib.o_copy_rectangle(self.wrap(src), self.wrap(dst), r, pt)

    def center_image(self, src, dst, origin, size):
        self.lib.o_center_image(self.wrap(src), self.wrap(dst), origin, size)

    def stretch_and_replace(self, h, size, interp):
        return self._replace(self.lib.o_stretch_and_replace, h, size, interp)

    def resize_and_replace(self, h, size, interp):
        return self._replace(self.lib.o_resize_and_replace, h, size, interp)

    def flip_rotate_90(self, h, direction):
        return self._replace(self.lib.o_flip_rotate_90, h, direction)

    def shift_image(self, h, delta):
        return self._replace(self.lib.o_shift_image, h, delta)

    def mirror(self, h, direction):
        self.lib.o_mirror(self.wrap(h), direction)

    def apply_masks(self, h, masks, color):
        arr = (A.Rectangle * max(1, len(masks)))(*masks)
        self.lib.o_apply_masks(self.wrap(h), arr, len(masks), color)

    def apply_wipes(self, h, wipes, color):
        self.lib.o_apply_wipes(self.wrap(h), C.byref(wipes), color)

    def apply_border(self, h, border, color):
        self.lib.o_apply_border(self.wrap(h), border, color)

    def detect_masks(self, h, params, points):
        pts = (A.Point * max(1, len(points)))(*points)
        masks = (A.Rectangle * max(1, len(points)))()
        n = self.lib.o_detect_masks(self.wrap(h), C.byref(params), pts, len(points), masks)
        return n, [masks[i] for i in range(len(points))]

    def align_mask(self, h, inside, outside, params):
        self.lib.o_align_mask(self.wrap(h), inside, outside, params)

    def detect_border(self, h, params, outside):
        return self.lib.o_detect_border(self.wrap(h), params, outside)

    def blackfilter(self, h, params):
        self.lib.o_blackfilter(self.wrap(h), C.byref(params))

    def blurfilter(self, h, params, white):
        self.lib.o_blurfilter(self.wrap(h), params, white)

    def noisefilter(self, h, intensity, white):
        self.lib.o_noisefilter(self.wrap(h), intensity, white)

    def grayfilter(self, h, params):
        self.lib.o_grayfilter(self.wrap(h), params)

    def detect_rotation(self, h, mask, params):
        return self.lib.o_detect_rotation(self.wrap(h), mask, C.byref(params))

    def rotation_peaks(self, h, mask, params):
        out = np.zeros(4 * 1024, np.int32)
        n = self.lib.o_rotation_peaks(self.wrap(h), mask, C.byref(params), out.ctypes.data, out.size)
        assert n >= 0
        return out[:n].copy()

    def deskew(self, h, mask, radians, interp):
        self.lib.o_deskew(self.wrap(h), mask, radians, interp)

    def center_mask(self, h, center, area):
        self.lib.o_center_mask(self.wrap(h), center, area)

    # -- pipeline ----------------------------------------------------------
    def process_sheet(self, options, pages):
        """Returns (sheet HostImage [RGB24], output_format, SheetReport)."""
        n = int(options.input_count)
        arr = (OImage * max(1, n))()
        for j in range(n):
            if j < len(pages) and pages[j] is not None:
                arr[j] = self.wrap(pages[j])
        out = OImage()
        fmt = C.c_int32()
        rep = A.SheetReport()
        rc = self.lib.o_process_sheet(C.byref(options), arr, C.byref(out), C.byref(fmt),
                                      C.byref(rep))
        if rc != 0:
            raise RuntimeError("oracle process_sheet failed (%d)" % rc)
        return self.adopt(out), fmt.value, rep

    def convert_for_save(self, sheet, fmt):
        return self.adopt(self.lib.o_convert_for_save(self.wrap(sheet), fmt))

    def stats(self):
        s = OStats()
        self.lib.o_stats_get(C.byref(s))
        return {n: getattr(s, n) for n, _ in OStats._fields_}

    def stats_reset(self):
        self.lib.o_stats_reset()
