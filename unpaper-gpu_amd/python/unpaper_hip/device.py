"""ctypes binding of libunpaper_hip.so (the HIP backend's C ABI).

Mirrors the reference's operator interface: `Backend` exposes the 20
`ImageBackend` ops (imageprocess/backend.h:22-56) under the same names and
argument meaning, operating on `DeviceImage` (Image{AVFrame*,...} peer,
image.h:11-15).  Errors raised by the library surface as `UnpaperHipError`.
There is no fallback: if the library or a GPU is missing, construction fails.
"""
import ctypes as C
import os

import numpy as np

from . import ctypes_abi as A
from .hostimage import HostImage, min_linesize

_PKG = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# UNPAPER_HIP_LIB selects another build of the same library (the `make lib
# DIAG=1` tuning build); uphip_version() names a diagnostics build.
LIB_PATH = os.environ.get("UNPAPER_HIP_LIB") or os.path.join(_PKG, "lib", "libunpaper_hip.so")

# every function the header declares (include/unpaper_hip.h)
EXPORTED = [
    "uphip_create_image", "uphip_free_image", "uphip_replace_image",
    "uphip_create_compatible_image", "uphip_size_of_image", "uphip_image_format",
    "uphip_image_upload", "uphip_image_download", "uphip_image_device_ptr",
    "uphip_image_device_pitch", "uphip_wipe_rectangle", "uphip_copy_rectangle",
    "uphip_center_image", "uphip_stretch_and_replace", "uphip_resize_and_replace",
    "uphip_flip_rotate_90", "uphip_mirror", "uphip_shift_image", "uphip_apply_masks",
    "uphip_apply_wipes", "uphip_apply_border", "uphip_detect_masks", "uphip_align_mask",
    "uphip_detect_border", "uphip_blackfilter", "uphip_blurfilter", "uphip_noisefilter",
    "uphip_grayfilter", "uphip_detect_rotation", "uphip_deskew", "uphip_backend",
    "uphip_try_init", "uphip_init_status_string", "uphip_device_count", "uphip_set_device",
    "uphip_get_device", "uphip_stream_acquire", "uphip_stream_release",
    "uphip_set_current_stream", "uphip_stream_forget", "uphip_get_current_stream",
    "uphip_synchronize",
    "uphip_last_error", "uphip_clear_error", "uphip_set_fatal_errors", "uphip_version",
    "uphip_abi_sizeof", "uphip_abi_offsetof",
    "uphip_options_init", "uphip_batch_create", "uphip_batch_destroy",
    "uphip_batch_output_info", "uphip_batch_input_ptr", "uphip_batch_set_input",
    "uphip_batch_run_device", "uphip_batch_run", "uphip_batch_wait",
    "uphip_batch_get_output", "uphip_batch_output_ptr", "uphip_batch_get_report",
    "uphip_batch_kernel_times", "uphip_batch_set_timing", "uphip_synth_pages", "uphip_synth_page_host",
    "uphip_synth_sheets_rgb", "uphip_synth_sheet_rgb_host",
    "uphip_device_alloc", "uphip_device_free", "uphip_memcpy_htod", "uphip_memcpy_dtoh",
    "uphip_batch_upload_async", "uphip_batch_download_async", "uphip_batch_query",
    "uphip_batch_stream", "uphip_batch_output_pitch", "uphip_pnm_probe", "uphip_pnm_read", "uphip_pnm_write",
    "uphip_png_probe", "uphip_png_read", "uphip_image_probe", "uphip_image_read",
    "uphip_source_callback", "uphip_source_memory", "uphip_source_pnm", "uphip_source_destroy",
    "uphip_sink_callback", "uphip_sink_memory", "uphip_sink_pnm", "uphip_sink_discard",
    "uphip_sink_destroy", "uphip_runner_create", "uphip_runner_destroy",
    "uphip_runner_run_device", "uphip_runner_run_host", "uphip_runner_get_stats",
    "uphip_runner_output_info", "uphip_runner_batch", "uphip_runner_layout", "uphip_batch_device_bytes", "uphip_host_alloc", "uphip_host_free",
    "uphip_check_libm", "uphip_jpeg_probe", "uphip_jpeg_read", "uphip_jpeg_decode",
    "uphip_jpeg_entropy_decode", "uphip_runner_placement", "uphip_runner_slot_chunk",
    "uphip_jpeg_encode", "uphip_batch_encode_jpeg_async", "uphip_batch_jpeg_sizes",
    "uphip_batch_jpeg_download_async", "uphip_batch_jpeg_page", "uphip_sink_jpeg",
    "uphip_detect_rotation_peaks", "uphip_jp2_probe", "uphip_jp2_read", "uphip_jp2_decode",
    "uphip_jp2_encode", "uphip_sink_jp2", "uphip_jp2_entropy_decode",
    "uphip_pdf_open", "uphip_pdf_open_memory", "uphip_pdf_close", "uphip_pdf_page_count",
    "uphip_pdf_needs_password", "uphip_pdf_get_page_info", "uphip_pdf_extract_page_image",
    "uphip_pdf_free_image", "uphip_pdf_get_metadata", "uphip_pdf_free_metadata",
    "uphip_pdf_image_format_name", "uphip_pdf_is_pdf_file", "uphip_pdf_page_probe",
    "uphip_pdf_read_page", "uphip_pdf_writer_create", "uphip_pdf_writer_add_page_jpeg",
    "uphip_pdf_writer_add_page_jp2", "uphip_pdf_writer_add_page_pixels",
    "uphip_pdf_writer_page_count", "uphip_pdf_writer_close", "uphip_pdf_writer_abort",
    "uphip_source_pdf", "uphip_source_page_count", "uphip_sink_pdf", "uphip_sink_finish",
    "uphip_jbig2_decode", "uphip_jbig2_free_image",
]


class UnpaperHipError(RuntimeError):
    pass


class Image(C.Structure):
    _fields_ = [("frame", C.c_void_p), ("background", A.Pixel), ("abs_black_threshold", C.c_uint8)]


_lib = None


def load_library(path=LIB_PATH):
    """Load the library (no GPU needed to load; ops need one)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise UnpaperHipError("libunpaper_hip.so not built (run `make lib`): " + path)
    L = C.CDLL(path)
    pim = C.POINTER(Image)
    sig = {
        "uphip_create_image": (Image, [A.RectangleSize, C.c_int, C.c_bool, A.Pixel, C.c_uint8]),
        "uphip_free_image": (None, [pim]),
        "uphip_size_of_image": (A.RectangleSize, [Image]),
        "uphip_image_format": (C.c_int, [Image]),
        "uphip_image_upload": (C.c_int, [Image, C.c_void_p, C.c_int64]),
        "uphip_image_download": (C.c_int, [Image, C.c_void_p, C.c_int64]),
        "uphip_image_device_ptr": (C.c_void_p, [Image]),
        "uphip_image_device_pitch": (C.c_int64, [Image]),
        "uphip_wipe_rectangle": (None, [Image, A.Rectangle, A.Pixel]),
        "uphip_copy_rectangle": (None, [Image, Image, A.Rectangle, A.Point]),
        "uphip_center_image": (None, [Image, Image, A.Point, A.RectangleSize]),
        "uphip_stretch_and_replace": (None, [pim, A.RectangleSize, C.c_int]),
        "uphip_resize_and_replace": (None, [pim, A.RectangleSize, C.c_int]),
        "uphip_flip_rotate_90": (None, [pim, C.c_int8]),
        "uphip_mirror": (None, [Image, A.Direction]),
        "uphip_shift_image": (None, [pim, A.Delta]),
        "uphip_apply_masks": (None, [Image, C.POINTER(A.Rectangle), C.c_size_t, A.Pixel]),
        "uphip_apply_wipes": (None, [Image, A.Wipes, A.Pixel]),
        "uphip_apply_border": (None, [Image, A.Border, A.Pixel]),
        "uphip_detect_masks": (C.c_size_t, [Image, A.MaskDetectionParameters,
                                            C.POINTER(A.Point), C.c_size_t,
                                            C.POINTER(A.Rectangle)]),
        "uphip_align_mask": (None, [Image, A.Rectangle, A.Rectangle, A.MaskAlignmentParameters]),
        "uphip_detect_border": (A.Border, [Image, A.BorderScanParameters, A.Rectangle]),
        "uphip_blackfilter": (None, [Image, A.BlackfilterParameters]),
        "uphip_blurfilter": (None, [Image, A.BlurfilterParameters, C.c_uint8]),
        "uphip_noisefilter": (None, [Image, C.c_uint64, C.c_uint8]),
        "uphip_grayfilter": (None, [Image, A.GrayfilterParameters]),
        "uphip_detect_rotation": (C.c_float, [Image, A.Rectangle, A.DeskewParameters]),
        "uphip_detect_rotation_peaks": (C.c_int32, [Image, A.Rectangle, A.DeskewParameters,
                                                    C.c_void_p, C.c_int32]),
        "uphip_deskew": (None, [Image, A.Rectangle, C.c_float, C.c_int]),
        "uphip_try_init": (C.c_int, []),
        "uphip_init_status_string": (C.c_char_p, [C.c_int]),
        "uphip_device_count": (C.c_int, []),
        "uphip_set_device": (C.c_int, [C.c_int]),
        "uphip_get_device": (C.c_int, []),
        "uphip_synchronize": (C.c_int, []),
        "uphip_stream_forget": (None, [C.c_void_p]),
        "uphip_last_error": (C.c_char_p, []),
        "uphip_clear_error": (None, []),
        "uphip_set_fatal_errors": (None, [C.c_bool]),
        "uphip_version": (C.c_char_p, []),
        "uphip_options_init": (None, [C.POINTER(A.Options)]),
        "uphip_abi_sizeof": (C.c_size_t, [C.c_char_p]),
        "uphip_abi_offsetof": (C.c_size_t, [C.c_char_p, C.c_char_p]),
        "uphip_batch_create": (C.c_void_p, [C.POINTER(A.Options), C.POINTER(A.BatchGeometry)]),
        "uphip_batch_destroy": (None, [C.c_void_p]),
        "uphip_batch_output_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32),
                                              C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                              C.POINTER(C.c_int64)]),
        "uphip_batch_input_ptr": (C.c_void_p, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]),
        "uphip_batch_set_input": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64]),
        "uphip_batch_run_device": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64,
                                             C.c_int64]),
        "uphip_batch_run": (C.c_int, [C.c_void_p, C.c_int32]),
        "uphip_batch_wait": (C.c_int, [C.c_void_p]),
        "uphip_batch_get_output": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64]),
        "uphip_batch_output_ptr": (C.c_void_p, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64)]),
        "uphip_batch_get_report": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(A.SheetReport)]),
        "uphip_batch_set_timing": (C.c_int, [C.c_void_p, C.c_int32]),
        "uphip_batch_kernel_times": (C.c_int, [C.c_void_p, C.POINTER(C.c_char_p),
                                               C.POINTER(C.c_float), C.c_int]),
        "uphip_synth_pages": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int32, C.c_int32,
                                        C.c_uint32, C.c_int32]),
        "uphip_synth_page_host": (None, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                         C.c_uint32]),
        "uphip_batch_upload_async": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int64,
                                               C.c_int64]),
        "uphip_batch_download_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64]),
        "uphip_batch_query": (C.c_int, [C.c_void_p]),
        "uphip_batch_stream": (C.c_void_p, [C.c_void_p]),
        "uphip_batch_output_pitch": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
        "uphip_pnm_probe": (C.c_int, [C.c_char_p, C.POINTER(A.PnmInfo)]),
        "uphip_pnm_read": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.POINTER(A.PnmInfo)]),
        "uphip_png_probe": (C.c_int, [C.c_char_p, C.POINTER(A.PnmInfo)]),
        "uphip_png_read": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.POINTER(A.PnmInfo)]),
        "uphip_image_probe": (C.c_int, [C.c_char_p, C.POINTER(A.PnmInfo)]),
        "uphip_image_read": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.POINTER(A.PnmInfo)]),
        "uphip_pnm_write": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                      C.c_int32]),
        "uphip_source_callback": (C.c_void_p, [A.LoadFn, C.c_void_p]),
        "uphip_source_memory": (C.c_void_p, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64]),
        "uphip_source_pnm": (C.c_void_p, [C.POINTER(C.c_char_p), C.c_int64]),
        "uphip_source_destroy": (None, [C.c_void_p]),
        "uphip_sink_callback": (C.c_void_p, [A.StoreFn, C.c_void_p]),
        "uphip_sink_memory": (C.c_void_p, [C.c_void_p, C.c_int64, C.c_int64, C.c_int64]),
        "uphip_sink_pnm": (C.c_void_p, [C.c_char_p, C.c_int64]),
        "uphip_sink_discard": (C.c_void_p, []),
        "uphip_sink_destroy": (None, [C.c_void_p]),
        "uphip_runner_create": (C.c_void_p, [C.POINTER(A.Options), C.POINTER(A.BatchGeometry),
                                             C.POINTER(A.RunnerConfig)]),
        "uphip_runner_destroy": (None, [C.c_void_p]),
        "uphip_runner_run_device": (C.c_int, [C.c_void_p, C.POINTER(A.DevicePages), C.c_int32]),
        "uphip_runner_run_host": (C.c_int, [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]),
        "uphip_runner_get_stats": (C.c_int, [C.c_void_p, C.POINTER(A.RunnerStats)]),
        "uphip_runner_layout": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                          C.POINTER(C.c_int64)]),
        "uphip_batch_device_bytes": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64)]),
        "uphip_runner_output_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32),
                                               C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                               C.POINTER(C.c_int64)]),
        "uphip_runner_batch": (C.c_void_p, [C.c_void_p, C.c_int32, C.c_int32]),
        "uphip_runner_slot_chunk": (C.c_int64, [C.c_void_p, C.c_int32, C.c_int32,
                                                C.POINTER(C.c_int32)]),
        "uphip_host_alloc": (C.c_void_p, [C.c_size_t]),
        "uphip_host_free": (None, [C.c_void_p]),
        "uphip_synth_sheets_rgb": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_int32,
                                             C.c_int32, C.c_uint32, C.c_int32]),
        "uphip_synth_sheet_rgb_host": (None, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32,
                                              C.c_uint32]),
        "uphip_device_alloc": (C.c_void_p, [C.c_size_t]),
        "uphip_device_free": (None, [C.c_void_p]),
        "uphip_memcpy_htod": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
        "uphip_memcpy_dtoh": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
        "uphip_check_libm": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint64)]),
        "uphip_runner_placement": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int32),
                                             C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
        "uphip_jpeg_probe": (C.c_int, [C.c_char_p, C.POINTER(A.PnmInfo)]),
        "uphip_jpeg_read": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.POINTER(A.PnmInfo)]),
        "uphip_jpeg_decode": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64,
                                        C.POINTER(A.PnmInfo)]),
        "uphip_jpeg_entropy_decode": (C.c_int64, [C.c_void_p, C.c_size_t, C.c_void_p,
                                                  C.c_int64]),
        "uphip_jpeg_encode": (C.c_int64, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                          C.c_int32, C.c_int32, C.c_void_p, C.c_int64]),
        "uphip_batch_encode_jpeg_async": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
        "uphip_batch_jpeg_sizes": (C.c_int64, [C.c_void_p, C.POINTER(C.c_int64), C.c_int32]),
        "uphip_batch_jpeg_download_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
        "uphip_batch_jpeg_page": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p),
                                            C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                            C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
        "uphip_sink_jpeg": (C.c_void_p, [C.c_char_p, C.c_int64, C.c_int32, C.c_int32]),
        "uphip_jp2_probe": (C.c_int, [C.c_char_p, C.POINTER(A.PnmInfo)]),
        "uphip_jp2_read": (C.c_int, [C.c_char_p, C.c_void_p, C.c_int64, C.POINTER(A.PnmInfo)]),
        "uphip_jp2_decode": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64,
                                       C.POINTER(A.PnmInfo)]),
        "uphip_jp2_encode": (C.c_int64, [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_void_p, C.c_int64]),
        "uphip_sink_jp2": (C.c_void_p, [C.c_char_p, C.c_int64]),
        "uphip_jp2_entropy_decode": (C.c_int64, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int64,
                                                 C.POINTER(A.PnmInfo)]),
        "uphip_pdf_open": (C.c_void_p, [C.c_char_p]),
        "uphip_pdf_open_memory": (C.c_void_p, [C.c_void_p, C.c_size_t]),
        "uphip_pdf_close": (None, [C.c_void_p]),
        "uphip_pdf_page_count": (C.c_int, [C.c_void_p]),
        "uphip_pdf_needs_password": (C.c_int, [C.c_void_p]),
        "uphip_pdf_get_page_info": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(A.PdfPageInfo)]),
        "uphip_pdf_extract_page_image": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(A.PdfImage)]),
        "uphip_pdf_free_image": (None, [C.POINTER(A.PdfImage)]),
        "uphip_pdf_get_metadata": (C.c_int, [C.c_void_p, C.POINTER(A.PdfMetadata)]),
        "uphip_pdf_free_metadata": (None, [C.POINTER(A.PdfMetadata)]),
        "uphip_pdf_image_format_name": (C.c_char_p, [C.c_int32]),
        "uphip_pdf_is_pdf_file": (C.c_int, [C.c_char_p]),
        "uphip_pdf_page_probe": (C.c_int, [C.c_void_p, C.c_int, C.c_int32, C.POINTER(A.PnmInfo)]),
        "uphip_pdf_read_page": (C.c_int, [C.c_void_p, C.c_int, C.c_int32, C.c_void_p, C.c_int64,
                                          C.POINTER(A.PnmInfo)]),
        "uphip_pdf_writer_create": (C.c_void_p, [C.c_char_p, C.POINTER(A.PdfMetadata), C.c_int32]),
        "uphip_pdf_writer_add_page_jpeg": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t,
                                                     C.c_int32, C.c_int32, C.c_int32]),
        "uphip_pdf_writer_add_page_jp2": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t,
                                                    C.c_int32, C.c_int32, C.c_int32]),
        "uphip_pdf_writer_add_page_pixels": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                                       C.c_int32, C.c_int32, C.c_int32]),
        "uphip_pdf_writer_page_count": (C.c_int, [C.c_void_p]),
        "uphip_pdf_writer_close": (C.c_int, [C.c_void_p]),
        "uphip_pdf_writer_abort": (None, [C.c_void_p]),
        "uphip_source_pdf": (C.c_void_p, [C.c_char_p, C.c_int32]),
        "uphip_source_page_count": (C.c_int64, [C.c_void_p]),
        "uphip_sink_pdf": (C.c_void_p, [C.c_char_p, C.POINTER(A.PdfMetadata), C.c_int32, C.c_int32,
                                        C.c_int32]),
        "uphip_sink_finish": (C.c_int, [C.c_void_p]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(L):
    e = L.uphip_last_error()
    if e is not None:
        L.uphip_clear_error()
        raise UnpaperHipError(e.decode())


class DeviceImage:
    """A frame resident in HBM (Image peer); freed on close()/GC."""

    def __init__(self, lib, img: Image):
        self.lib = lib
        self.img = img

    @classmethod
    def create(cls, lib, width, height, fmt, fill=False, background=(255, 255, 255),
               abs_black_threshold=170):
        img = lib.uphip_create_image(A.RectangleSize(width, height), fmt, fill,
                                     A.Pixel(*background), abs_black_threshold)
        _check(lib)
        if not img.frame:
            raise UnpaperHipError("create_image failed")
        return cls(lib, img)

    @classmethod
    def from_host(cls, lib, h: HostImage):
        d = cls.create(lib, h.width, h.height, h.format, False, h.background,
                       h.abs_black_threshold)
        arr = np.ascontiguousarray(h.data)
        lib.uphip_image_upload(d.img, arr.ctypes.data, arr.shape[1])
        _check(lib)
        return d

    @property
    def size(self):
        s = self.lib.uphip_size_of_image(self.img)
        return s.width, s.height

    @property
    def format(self):
        return self.lib.uphip_image_format(self.img)

    def to_host(self) -> HostImage:
        w, h = self.size
        fmt = self.format
        out = HostImage(w, h, fmt, background=(self.img.background.r, self.img.background.g,
                                               self.img.background.b),
                        abs_black_threshold=self.img.abs_black_threshold)
        self.lib.uphip_image_download(self.img, out.data.ctypes.data, out.linesize)
        _check(self.lib)
        return out

    def close(self):
        if self.img.frame:
            self.lib.uphip_free_image(C.byref(self.img))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Backend:
    """The HIP `ImageBackend` (backend.h:19-57) as Python methods."""

    name = "hip"

    def __init__(self, path=LIB_PATH):
        self.lib = L = load_library(path)
        st = L.uphip_try_init()
        if st != 0:
            raise UnpaperHipError("HIP backend unavailable: " +
                                  L.uphip_init_status_string(st).decode())

    def _done(self):
        _check(self.lib)

    def upload(self, h):
        return DeviceImage.from_host(self.lib, h)

    def create_image(self, width, height, fmt, fill=False, background=(255, 255, 255),
                     abs_black_threshold=170):
        return DeviceImage.create(self.lib, width, height, fmt, fill, background,
                                  abs_black_threshold)

    # -- ops ----------------------------------------------------------------
    def wipe_rectangle(self, d, r, color):
        self.lib.uphip_wipe_rectangle(d.img, r, color); self._done()

    def copy_rectangle(self, src, dst, r, pt):
        self.lib.uphip_copy_rectangle(src.img, dst.img, r, pt); self._done()

    def center_image(self, src, dst, origin, size):
        self.lib.uphip_center_image(src.img, dst.img, origin, size); self._done()

    def stretch_and_replace(self, d, size, interp):
        self.lib.uphip_stretch_and_replace(C.byref(d.img), size, interp); self._done()

    def resize_and_replace(self, d, size, interp):
        self.lib.uphip_resize_and_replace(C.byref(d.img), size, interp); self._done()

    def flip_rotate_90(self, d, direction):
        self.lib.uphip_flip_rotate_90(C.byref(d.img), direction); self._done()

    def mirror(self, d, direction):
        self.lib.uphip_mirror(d.img, direction); self._done()

    def shift_image(self, d, delta):
        self.lib.uphip_shift_image(C.byref(d.img), delta); self._done()

    def apply_masks(self, d, masks, color):
        arr = (A.Rectangle * max(1, len(masks)))(*masks)
        self.lib.uphip_apply_masks(d.img, arr, len(masks), color); self._done()

    def apply_wipes(self, d, wipes, color):
        self.lib.uphip_apply_wipes(d.img, wipes, color); self._done()

    def apply_border(self, d, border, color):
        self.lib.uphip_apply_border(d.img, border, color); self._done()

    def detect_masks(self, d, params, points):
        pts = (A.Point * max(1, len(points)))(*points)
        masks = (A.Rectangle * max(1, len(points)))()
        n = self.lib.uphip_detect_masks(d.img, params, pts, len(points), masks)
        self._done()
        return n, [masks[i] for i in range(len(points))]

    def align_mask(self, d, inside, outside, params):
        self.lib.uphip_align_mask(d.img, inside, outside, params); self._done()

    def detect_border(self, d, params, outside):
        b = self.lib.uphip_detect_border(d.img, params, outside); self._done()
        return b

    def blackfilter(self, d, params):
        self.lib.uphip_blackfilter(d.img, params); self._done()

    def blurfilter(self, d, params, white):
        self.lib.uphip_blurfilter(d.img, params, white); self._done()

    def noisefilter(self, d, intensity, white):
        self.lib.uphip_noisefilter(d.img, intensity, white); self._done()

    def grayfilter(self, d, params):
        self.lib.uphip_grayfilter(d.img, params); self._done()

    def detect_rotation_peaks(self, d, mask, params):
        """Per (edge, angle) peaks (uphip_detect_rotation_peaks) as an int32 array."""
        out = np.zeros(4 * 1024, np.int32)
        n = self.lib.uphip_detect_rotation_peaks(d.img, mask, params, out.ctypes.data, out.size)
        self._done()
        if n < 0:
            raise UnpaperHipError("detect_rotation_peaks failed")
        return out[:n].copy()

    def detect_rotation(self, d, mask, params):
        r = self.lib.uphip_detect_rotation(d.img, mask, params); self._done()
        return r

    def deskew(self, d, mask, radians, interp):
        self.lib.uphip_deskew(d.img, mask, radians, interp); self._done()

    def synchronize(self):
        self.lib.uphip_synchronize(); self._done()

    def default_options(self):
        o = A.Options()
        self.lib.uphip_options_init(C.byref(o))
        return o
