"""Batch sheet pipeline (uphip_batch_*): the device peer of process_sheet
(sheet_process.c:134) run by lib/batch_worker.c for every job, here for a whole
batch of sheets per launch sequence."""
import ctypes as C

import numpy as np

from . import ctypes_abi as A
from .device import UnpaperHipError, _check, load_library
from .hostimage import HostImage


def synth_page_host(width, height, page):
    """Deterministic synthetic GRAY8 page, host copy."""
    L = load_library()
    arr = np.empty((height, width), np.uint8)
    L.uphip_synth_page_host(arr.ctypes.data, width, width, height, page)
    return arr


class DeviceBuffer:
    """Raw HBM allocation (bench inputs)."""

    def __init__(self, nbytes):
        self.lib = load_library()
        self.ptr = self.lib.uphip_device_alloc(nbytes)
        _check(self.lib)
        if not self.ptr:
            raise UnpaperHipError("device_alloc failed")
        self.nbytes = nbytes

    def close(self):
        if self.ptr:
            self.lib.uphip_device_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    def __init__(self, options, capacity, page_width, page_height, page_format, timing=False):
        self.lib = L = load_library()
        self.options = options
        self.geometry = A.BatchGeometry(capacity, page_width, page_height, page_format)
        self.capacity = capacity
        self.handle = L.uphip_batch_create(C.byref(options), C.byref(self.geometry))
        _check(L)
        if not self.handle:
            raise UnpaperHipError("batch_create failed")
        w, h, f, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        L.uphip_batch_output_info(self.handle, C.byref(w), C.byref(h), C.byref(f), C.byref(n))
        if timing:
            self.set_timing(True)
        self.out_width, self.out_height, self.out_format = w.value, h.value, f.value

    def set_input(self, sheet, page_index, h: HostImage):
        slot = sheet * self.options.input_count + page_index
        arr = np.ascontiguousarray(h.data)
        if self.lib.uphip_batch_set_input(self.handle, slot, arr.ctypes.data, arr.shape[1]) != 0:
            _check(self.lib)

    def run(self, count):
        rc = self.lib.uphip_batch_run(self.handle, count)
        _check(self.lib)
        if rc != 0:
            raise UnpaperHipError("batch_run failed")

    def run_device(self, count, pages_ptr, pitch, page_stride):
        rc = self.lib.uphip_batch_run_device(self.handle, count, pages_ptr, pitch, page_stride)
        _check(self.lib)
        if rc != 0:
            raise UnpaperHipError("batch_run_device failed")

    def wait(self):
        rc = self.lib.uphip_batch_wait(self.handle)
        _check(self.lib)
        if rc != 0:
            raise UnpaperHipError("batch_wait failed")

    def output(self, sheet, background=(255, 255, 255), threshold=170) -> HostImage:
        out = HostImage(self.out_width, self.out_height, self.out_format, background=background,
                        abs_black_threshold=threshold)
        if self.lib.uphip_batch_get_output(self.handle, sheet, out.data.ctypes.data,
                                           out.linesize) != 0:
            _check(self.lib)
            raise UnpaperHipError("batch_get_output failed")
        return out

    def report(self, sheet):
        r = A.SheetReport()
        self.lib.uphip_batch_get_report(self.handle, sheet, C.byref(r))
        return r

    def set_timing(self, enable=True):
        """Record per-stage HIP events on every run (uphip_batch_set_timing)."""
        self.lib.uphip_batch_set_timing(self.handle, 1 if enable else 0)

    def stage_times(self):
        names = (C.c_char_p * 64)()
        ms = (C.c_float * 64)()
        n = self.lib.uphip_batch_kernel_times(self.handle, names, ms, 64)
        return [(names[i].decode(), ms[i]) for i in range(max(n, 0))]

    def close(self):
        if self.handle:
            self.lib.uphip_batch_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
