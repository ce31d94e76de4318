"""ctypes mirror of include/unpaper_hip.h (value types, options, report).

Field order and types follow the header exactly; `tests/test_abi.py` checks the
sizes against the C compiler's view (via `uphip_abi_sizeof` in the library and
`oracle_abi_sizeof` in the oracle build).
"""
import ctypes as C

MAX_MASKS = 100
MAX_POINTS = 100
MAX_PAGES = 2

FMT_NONE, FMT_GRAY8, FMT_Y400A, FMT_RGB24, FMT_MONOWHITE, FMT_MONOBLACK = -1, 0, 1, 2, 3, 4
INTERP_NN, INTERP_LINEAR, INTERP_CUBIC = 0, 1, 2
LAYOUT_NONE, LAYOUT_SINGLE, LAYOUT_DOUBLE = 0, 1, 2

NO_BLACKFILTER = 1 << 0
NO_NOISEFILTER = 1 << 1
NO_BLURFILTER = 1 << 2
NO_GRAYFILTER = 1 << 3
NO_MASK_SCAN = 1 << 4
NO_MASK_CENTER = 1 << 5
NO_DESKEW = 1 << 6
NO_WIPE = 1 << 7
NO_BORDER = 1 << 8
NO_BORDER_SCAN = 1 << 9
NO_BORDER_ALIGN = 1 << 10
NO_PROCESSING = (1 << 11) - 1   # "-n": every isExcluded() stage off


class Point(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32)]


class Delta(C.Structure):
    _fields_ = [("horizontal", C.c_int32), ("vertical", C.c_int32)]


class Direction(C.Structure):
    _fields_ = [("horizontal", C.c_bool), ("vertical", C.c_bool)]


class Edges(C.Structure):
    _fields_ = [("left", C.c_bool), ("top", C.c_bool), ("right", C.c_bool), ("bottom", C.c_bool)]


class Pixel(C.Structure):
    _fields_ = [("r", C.c_uint8), ("g", C.c_uint8), ("b", C.c_uint8)]


class Rectangle(C.Structure):
    _fields_ = [("vertex", Point * 2)]

    @classmethod
    def make(cls, x0, y0, x1, y1):
        r = cls()
        r.vertex[0].x, r.vertex[0].y, r.vertex[1].x, r.vertex[1].y = x0, y0, x1, y1
        return r

    def tuple(self):
        return (self.vertex[0].x, self.vertex[0].y, self.vertex[1].x, self.vertex[1].y)


class RectangleSize(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32)]


class Border(C.Structure):
    _fields_ = [("left", C.c_int32), ("top", C.c_int32), ("right", C.c_int32), ("bottom", C.c_int32)]

    def tuple(self):
        return (self.left, self.top, self.right, self.bottom)


class Wipes(C.Structure):
    _fields_ = [("count", C.c_size_t), ("areas", Rectangle * MAX_MASKS)]


class _HV_u32(C.Structure):
    _fields_ = [("horizontal", C.c_uint32), ("vertical", C.c_uint32)]


class _HV_i32(C.Structure):
    _fields_ = [("horizontal", C.c_int32), ("vertical", C.c_int32)]


class _HV_f32(C.Structure):
    _fields_ = [("horizontal", C.c_float), ("vertical", C.c_float)]


class BlackfilterParameters(C.Structure):
    _fields_ = [
        ("scan_size", RectangleSize),
        ("scan_step", Delta),
        ("scan_depth", _HV_u32),
        ("scan_direction", Direction),
        ("abs_threshold", C.c_uint8),
        ("intensity", C.c_int32),
        ("exclusions_count", C.c_size_t),
        ("exclusions", Rectangle * MAX_MASKS),
    ]


class BlurfilterParameters(C.Structure):
    _fields_ = [("scan_size", RectangleSize), ("scan_step", Delta), ("intensity", C.c_float)]


class GrayfilterParameters(C.Structure):
    _fields_ = [("scan_size", RectangleSize), ("scan_step", Delta), ("abs_threshold", C.c_uint8)]


class MaskDetectionParameters(C.Structure):
    _fields_ = [
        ("scan_size", RectangleSize),
        ("scan_step", Delta),
        ("scan_depth", _HV_i32),
        ("scan_direction", Direction),
        ("scan_threshold", _HV_f32),
        ("minimum_width", C.c_int32),
        ("maximum_width", C.c_int32),
        ("minimum_height", C.c_int32),
        ("maximum_height", C.c_int32),
    ]


class MaskAlignmentParameters(C.Structure):
    _fields_ = [("alignment", Edges), ("margin", Delta)]


class BorderScanParameters(C.Structure):
    _fields_ = [
        ("scan_size", RectangleSize),
        ("scan_step", Delta),
        ("scan_threshold", _HV_i32),
        ("scan_direction", Direction),
    ]


class DeskewParameters(C.Structure):
    _fields_ = [
        ("deskewScanRangeRad", C.c_float),
        ("deskewScanStepRad", C.c_float),
        ("deskewScanDeviationRad", C.c_float),
        ("deskewScanSize", C.c_int),
        ("deskewScanDepth", C.c_float),
        ("scan_edges", Edges),
    ]


class Options(C.Structure):
    _fields_ = [
        ("layout", C.c_int32),
        ("input_count", C.c_int32),
        ("output_count", C.c_int32),
        ("output_pixel_format", C.c_int32),
        ("disable", C.c_uint32),
        ("pre_rotate", C.c_int16),
        ("post_rotate", C.c_int16),
        ("pre_mirror", Direction),
        ("post_mirror", Direction),
        ("pre_shift", Delta),
        ("post_shift", Delta),
        ("sheet_size", RectangleSize),
        ("page_size", RectangleSize),
        ("post_page_size", RectangleSize),
        ("stretch_size", RectangleSize),
        ("post_stretch_size", RectangleSize),
        ("pre_zoom_factor", C.c_float),
        ("post_zoom_factor", C.c_float),
        ("sheet_background", Pixel),
        ("mask_color", Pixel),
        ("abs_black_threshold", C.c_uint8),
        ("abs_white_threshold", C.c_uint8),
        ("pre_border", Border),
        ("border", Border),
        ("post_border", Border),
        ("pre_wipes", Wipes),
        ("wipes", Wipes),
        ("post_wipes", Wipes),
        ("deskew_parameters", DeskewParameters),
        ("mask_detection_parameters", MaskDetectionParameters),
        ("mask_alignment_parameters", MaskAlignmentParameters),
        ("border_scan_parameters", BorderScanParameters),
        ("interpolate_type", C.c_int32),
        ("grayfilter_parameters", GrayfilterParameters),
        ("blackfilter_parameters", BlackfilterParameters),
        ("blurfilter_parameters", BlurfilterParameters),
        ("noisefilter_intensity", C.c_uint64),
        ("pre_mask_count", C.c_size_t),
        ("pre_masks", Rectangle * MAX_MASKS),
        ("point_count", C.c_size_t),
        ("points", Point * MAX_POINTS),
        ("middle_wipe", C.c_int32 * 2),
    ]


class SheetReport(C.Structure):
    _fields_ = [
        ("mask_count", C.c_int32),
        ("masks", Rectangle * MAX_PAGES),
        ("rotation", C.c_float * MAX_PAGES),
        ("border_masks", Rectangle * MAX_PAGES),
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("flags", C.c_uint32),
    ]


class PnmInfo(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("format", C.c_int32)]


RUNNER_MAX_DEVICES = 16


class RunnerConfig(C.Structure):
    _fields_ = [
        ("ndevices", C.c_int32),
        ("devices", C.POINTER(C.c_int32)),
        ("batches_per_device", C.c_int32),
        ("host_threads", C.c_int32),
        ("timing", C.c_int32),
    ]


class DevicePages(C.Structure):
    _fields_ = [
        ("pages", C.c_void_p),
        ("pitch", C.c_int64),
        ("page_stride", C.c_int64),
        ("count", C.c_int64),
    ]


class RunnerStats(C.Structure):
    _fields_ = [
        ("jobs_done", C.c_int64),
        ("jobs_failed", C.c_int64),
        ("jobs_per_device", C.c_int64 * RUNNER_MAX_DEVICES),
        ("wall_s", C.c_double),
        ("load_s", C.c_double),
        ("store_s", C.c_double),
    ]


LoadFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64)
StoreFn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int32,
                      C.c_int32, C.c_int32)


class BatchGeometry(C.Structure):
    _fields_ = [
        ("capacity", C.c_int32),
        ("page_width", C.c_int32),
        ("page_height", C.c_int32),
        ("page_format", C.c_int32),
    ]


def rect(x0, y0, x1, y1):
    return Rectangle.make(x0, y0, x1, y1)


def pixel(r, g=None, b=None):
    if g is None:
        g = b = r
    return Pixel(r, g, b)


ABI_STRUCTS = {
    "UphipPoint": Point, "UphipDelta": Delta, "UphipDirection": Direction,
    "UphipEdges": Edges, "UphipPixel": Pixel, "UphipRectangle": Rectangle,
    "UphipRectangleSize": RectangleSize, "UphipBorder": Border, "UphipWipes": Wipes,
    "UphipBlackfilterParameters": BlackfilterParameters,
    "UphipBlurfilterParameters": BlurfilterParameters,
    "UphipGrayfilterParameters": GrayfilterParameters,
    "UphipMaskDetectionParameters": MaskDetectionParameters,
    "UphipMaskAlignmentParameters": MaskAlignmentParameters,
    "UphipBorderScanParameters": BorderScanParameters,
    "UphipDeskewParameters": DeskewParameters, "UphipOptions": Options,
    "UphipSheetReport": SheetReport, "UphipBatchGeometry": BatchGeometry,
}


# PDF container (include/unpaper_hip.h, pdf/pdf_reader.h:31-63 peers)
class PdfImage(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("size", C.c_size_t),
                ("width", C.c_int32), ("height", C.c_int32),
                ("components", C.c_int32), ("bits_per_component", C.c_int32),
                ("format", C.c_int32), ("is_mask", C.c_int32),
                ("jbig2_globals", C.POINTER(C.c_uint8)), ("jbig2_globals_size", C.c_size_t)]


class PdfMetadata(C.Structure):
    _fields_ = [(n, C.c_char_p) for n in ("title", "author", "subject", "keywords", "creator",
                                           "producer", "creation_date", "modification_date")]


class PdfPageInfo(C.Structure):
    _fields_ = [("width", C.c_float), ("height", C.c_float), ("rotation", C.c_int32)]
