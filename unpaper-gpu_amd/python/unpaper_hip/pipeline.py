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


def synth_sheet_rgb_host(width, height, sheet):
    """C4 synthetic RGB24 double-page sheet (synth.h synth_rgb_channel), host copy."""
    L = load_library()
    arr = np.empty((height, width, 3), np.uint8)
    L.uphip_synth_sheet_rgb_host(arr.ctypes.data, width * 3, width, height, sheet)
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
        # the copy is asynchronous on the batch stream: the source must live
        # until the stream has passed it (released by wait())
        self._inputs = getattr(self, "_inputs", {})
        self._inputs[slot] = arr
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
        self._inputs = {}
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

    def encode_jpeg(self, quality=0, sampling=0):
        """Queue the GPU JPEG output branch on the last run's pages
        (uphip_batch_encode_jpeg_async)."""
        if self.lib.uphip_batch_encode_jpeg_async(self.handle, quality, sampling) != 0:
            _check(self.lib)
            raise UnpaperHipError("batch_encode_jpeg failed")

    def jpeg_files(self, pages):
        """The encoded files of the last encode_jpeg (None for a page the
        batch's buffers could not hold: uphip_batch_jpeg_page + jpeg_encode)."""
        L = self.lib
        self.wait()
        sizes = (C.c_int64 * pages)()
        total = L.uphip_batch_jpeg_sizes(self.handle, sizes, pages)
        _check(L)
        buf = np.zeros(max(total, 1), np.uint8)
        if total > 0 and L.uphip_batch_jpeg_download_async(self.handle, buf.ctypes.data, total) != 0:
            _check(L)
        self.wait()
        out, off = [], 0
        for i in range(pages):
            n = sizes[i]
            if n > 0:
                out.append(buf[off:off + n].tobytes())
                off += n
            else:
                out.append(None)
        return out

    def jpeg_page(self, page):
        """(device pointer, pitch, width, height, format) of output page `page`."""
        src, pitch = C.c_void_p(), C.c_int64()
        w, h, f = C.c_int32(), C.c_int32(), C.c_int32()
        if self.lib.uphip_batch_jpeg_page(self.handle, page, C.byref(src), C.byref(pitch),
                                          C.byref(w), C.byref(h), C.byref(f)) != 0:
            _check(self.lib)
        return src.value, pitch.value, w.value, h.value, f.value

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


class HostBuffer:
    """Pinned host memory (uphip_host_alloc) viewed as a numpy uint8 array."""

    def __init__(self, nbytes):
        self.lib = load_library()
        self.ptr = self.lib.uphip_host_alloc(nbytes)
        _check(self.lib)
        if not self.ptr:
            raise UnpaperHipError("host_alloc failed")
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def close(self):
        if self.ptr:
            self.array = None
            self.lib.uphip_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Runner:
    """Multi-device runner (uphip_runner_*): the peer of lib/batch_worker.c's
    batch_process_parallel with one host thread and `streams` batches of
    `sheets` sheets per device; sources/sinks are the decode/encode queues.
    sheets=0 / streams=0: the runner sizes them from the geometry and the
    device's free memory (uphip_runner_layout reports the choice)."""

    def __init__(self, options, sheets, page_width, page_height, page_format, devices=(0,),
                 streams=4, host_threads=0, timing=False):
        self.lib = L = load_library()
        self.options = options
        self.geometry = A.BatchGeometry(sheets, page_width, page_height, page_format)
        self._devs = (C.c_int32 * len(devices))(*devices)
        self.config = A.RunnerConfig(len(devices), self._devs, streams, host_threads,
                                     1 if timing else 0)
        self.ndevices = len(devices)
        self.streams = streams
        self.handle = L.uphip_runner_create(C.byref(options), C.byref(self.geometry),
                                            C.byref(self.config))
        _check(L)
        if not self.handle:
            raise UnpaperHipError("runner_create failed")
        w, h, f, ls = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        L.uphip_runner_output_info(self.handle, C.byref(w), C.byref(h), C.byref(f), C.byref(ls))
        self.out_width, self.out_height, self.out_format = w.value, h.value, f.value
        self.out_linesize = ls.value
        k, cap, bb = C.c_int32(), C.c_int32(), C.c_int64()
        L.uphip_runner_layout(self.handle, C.byref(k), C.byref(cap), C.byref(bb))
        self.streams, self.batch_bytes = k.value, bb.value
        self.geometry.capacity = cap.value

    def batch(self, device_index, slot):
        """The Batch object behind one stream (borrowed; not closed here)."""
        h = self.lib.uphip_runner_batch(self.handle, device_index, slot)
        if not h:
            raise UnpaperHipError("no such batch")
        b = Batch.__new__(Batch)
        b.lib, b.options, b.capacity, b.handle = self.lib, self.options, self.geometry.capacity, h
        b.out_width, b.out_height, b.out_format = self.out_width, self.out_height, self.out_format
        b.close = lambda: None
        return b

    def slot_chunk(self, device_index, slot):
        """(first job, sheet count) of the chunk batch `slot` ran last (its
        outputs are resident), or None when it has run none."""
        n = C.c_int32(0)
        first = self.lib.uphip_runner_slot_chunk(self.handle, device_index, slot, C.byref(n))
        return None if first < 0 else (first, n.value)

    def run_device(self, shards, passes=1):
        """shards: one (device_ptr, pitch, page_stride, count) per device.
        Returns (failed jobs, the library's error message or None)."""
        arr = (A.DevicePages * self.ndevices)(*[A.DevicePages(*s) for s in shards])
        failed = self.lib.uphip_runner_run_device(self.handle, arr, passes)
        err = self.lib.uphip_last_error()
        self.lib.uphip_clear_error()
        return failed, (err.decode() if err else None)

    def run_host(self, njobs, source, sink):
        failed = self.lib.uphip_runner_run_host(self.handle, njobs, source.handle, sink.handle)
        err = self.lib.uphip_last_error()
        self.lib.uphip_clear_error()
        return failed, (err.decode() if err else None)

    def stats(self):
        s = A.RunnerStats()
        self.lib.uphip_runner_get_stats(self.handle, C.byref(s))
        return s

    def placement(self, device_index):
        """(NUMA node or -1, CPUs bound to or 0, load/store pool threads)."""
        node, ncpu, pool = C.c_int32(), C.c_int32(), C.c_int32()
        if self.lib.uphip_runner_placement(self.handle, device_index, C.byref(node),
                                           C.byref(ncpu), C.byref(pool)) != 0:
            _check(self.lib)
        return node.value, ncpu.value, pool.value

    def close(self):
        if self.handle:
            self.lib.uphip_runner_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Handle:
    def __init__(self, handle, destroy, keep=()):
        self.handle = handle
        self._destroy = destroy
        self._keep = keep          # buffers / callbacks the C side points into

    def close(self):
        if self.handle:
            self._destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def source_memory(ptr, linesize, page_stride, npages, keep=None):
    L = load_library()
    h = L.uphip_source_memory(ptr, linesize, page_stride, npages)
    _check(L)
    return _Handle(h, L.uphip_source_destroy, (keep,))


def source_pnm(paths):
    L = load_library()
    arr = (C.c_char_p * len(paths))(*[p.encode() for p in paths])
    h = L.uphip_source_pnm(arr, len(paths))
    _check(L)
    return _Handle(h, L.uphip_source_destroy, (arr,))


def source_pdf(path, dpi=0):
    """Page i of a PDF as input page i (uphip_source_pdf; dpi 0 = the page
    images as they are, dpi > 0 = the reference's size check)."""
    L = load_library()
    h = L.uphip_source_pdf(path.encode(), dpi)
    _check(L)
    if not h:
        raise UnpaperHipError("source_pdf failed")
    return _Handle(h, L.uphip_source_destroy)


def source_page_count(src):
    L = load_library()
    n = L.uphip_source_page_count(src.handle)
    _check(L)
    return n


def source_callback(fn):
    """fn(job, page, dst_ptr, linesize) -> 0 on success (called from C threads)."""
    L = load_library()
    cb = A.LoadFn(lambda user, job, page, dst, ls: fn(job, page, dst, ls))
    h = L.uphip_source_callback(cb, None)
    _check(L)
    return _Handle(h, L.uphip_source_destroy, (cb,))


def sink_memory(ptr, linesize, sheet_stride, nsheets, keep=None):
    L = load_library()
    h = L.uphip_sink_memory(ptr, linesize, sheet_stride, nsheets)
    _check(L)
    return _Handle(h, L.uphip_sink_destroy, (keep,))


def sink_pnm(pattern, wrap=0):
    L = load_library()
    h = L.uphip_sink_pnm(pattern.encode(), wrap)
    _check(L)
    return _Handle(h, L.uphip_sink_destroy)


def sink_jpeg(pattern, wrap=0, quality=0, sampling=0):
    """JPEG files encoded on the device (uphip_sink_jpeg; quality 0 = 85,
    sampling 0 = 4:4:4, 1 = 4:2:2, 2 = 4:2:0 for RGB24 sheets)."""
    L = load_library()
    h = L.uphip_sink_jpeg(pattern.encode(), wrap, quality, sampling)
    _check(L)
    return _Handle(h, L.uphip_sink_destroy)


def jpeg_encode(device_ptr, pitch, width, height, fmt, quality=0, sampling=0):
    """uphip_jpeg_encode: one device image -> JPEG file bytes."""
    L = load_library()
    n = L.uphip_jpeg_encode(device_ptr, pitch, width, height, fmt, quality, sampling, None, 0)
    _check(L)
    if n <= 0:
        raise UnpaperHipError("jpeg_encode failed")
    buf = np.zeros(n, np.uint8)
    m = L.uphip_jpeg_encode(device_ptr, pitch, width, height, fmt, quality, sampling,
                            buf.ctypes.data, n)
    _check(L)
    if m != n:
        raise UnpaperHipError("jpeg_encode: size changed between calls")
    return buf.tobytes()


def sink_jp2(pattern, wrap=0):
    """Lossless JPEG 2000 files (uphip_sink_jp2: transforms on the device,
    code-blocks on the store tasks)."""
    L = load_library()
    h = L.uphip_sink_jp2(pattern.encode(), wrap)
    _check(L)
    return _Handle(h, L.uphip_sink_destroy)


def jp2_encode(device_ptr, pitch, width, height, fmt):
    """uphip_jp2_encode: one device image -> lossless JP2 file bytes."""
    L = load_library()
    cap = width * height * (1 if fmt == 0 else 3) // 2 + 65536
    buf = np.zeros(cap, np.uint8)
    n = L.uphip_jp2_encode(device_ptr, pitch, width, height, fmt, buf.ctypes.data, cap)
    _check(L)
    if n > cap:
        buf = np.zeros(n, np.uint8)
        n = L.uphip_jp2_encode(device_ptr, pitch, width, height, fmt, buf.ctypes.data, n)
        _check(L)
    if n <= 0:
        raise UnpaperHipError("jp2_encode failed")
    return buf[:n].tobytes()


class _PdfSink(_Handle):
    def finish(self):
        """Completes the PDF (uphip_sink_finish)."""
        L = load_library()
        if self.handle and L.uphip_sink_finish(self.handle) != 0:
            _check(L)
            raise UnpaperHipError("sink_finish failed")


def sink_pdf(path, meta=None, dpi=0, quality=0, mode=0):
    """All output pages into one PDF (uphip_sink_pdf): mode 0 = JPEG pages
    (fast), 1 = lossless JPEG 2000 pages (high); dpi 0 = 300.  Call
    finish() after the run."""
    from .pdf import _meta_struct
    L = load_library()
    m, keep = _meta_struct(meta)
    h = L.uphip_sink_pdf(path.encode(), C.byref(m) if m is not None else None, dpi, quality, mode)
    _check(L)
    if not h:
        raise UnpaperHipError("sink_pdf failed")
    return _PdfSink(h, L.uphip_sink_destroy, (m, keep))


def sink_discard():
    L = load_library()
    return _Handle(L.uphip_sink_discard(), L.uphip_sink_destroy)


def pnm_write(path, h: HostImage):
    L = load_library()
    arr = np.ascontiguousarray(h.data)
    if L.uphip_pnm_write(path.encode(), arr.ctypes.data, arr.shape[1], h.width, h.height,
                         h.format) != 0:
        _check(L)


def pnm_read(path) -> HostImage:
    L = load_library()
    info = A.PnmInfo()
    if L.uphip_pnm_probe(path.encode(), C.byref(info)) != 0:
        _check(L)
    img = HostImage(info.width, info.height, info.format)
    if L.uphip_pnm_read(path.encode(), img.data.ctypes.data, img.linesize, C.byref(info)) != 0:
        _check(L)
    return img


def image_read(path) -> HostImage:
    """loadImage's peer (file.c:29-131): PNG or PNM, picked by signature."""
    L = load_library()
    info = A.PnmInfo()
    if L.uphip_image_probe(path.encode(), C.byref(info)) != 0:
        _check(L)
    img = HostImage(info.width, info.height, info.format)
    if L.uphip_image_read(path.encode(), img.data.ctypes.data, img.linesize, C.byref(info)) != 0:
        _check(L)
    return img
