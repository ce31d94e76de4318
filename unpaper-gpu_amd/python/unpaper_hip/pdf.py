"""PDF container: the reference's pdf/pdf_reader.h + pdf/pdf_writer.h surface
over the C ABI (csrc/pdf.cpp; MuPDF is not used).

    doc = PdfDocument.open("scan.pdf")          # pdf_open
    doc.page_count, doc.page_info(0)             # pdf_page_count, pdf_get_page_info
    img = doc.extract_page_image(0)              # pdf_extract_page_image
    pix = doc.read_page(0, dpi=0)                # decode: JPEG / JP2 on the device
    w = PdfWriter.create("out.pdf", meta, 300)   # pdf_writer_create
    w.add_page_jpeg(data, width, height); w.close()

Pages that need a rasteriser (vector / text content, or an image that does
not fill the page at the requested dpi), encrypted files and JBIG2 / CCITT
images raise UnpaperHipError with the cause.
"""
import ctypes as C
from dataclasses import dataclass
from typing import Optional

from . import ctypes_abi as A
from .device import UnpaperHipError, _check, load_library
from .hostimage import HostImage

IMAGE_UNKNOWN, IMAGE_JPEG, IMAGE_JP2, IMAGE_JBIG2, IMAGE_CCITT, IMAGE_PNG, IMAGE_RAW, IMAGE_FLATE = range(8)
PIXEL_GRAY8, PIXEL_RGB24 = 0, 1
META_FIELDS = ("title", "author", "subject", "keywords", "creator", "producer",
               "creation_date", "modification_date")


def _fail(L, what):
    _check(L)
    raise UnpaperHipError(what)


@dataclass
class PdfImage:
    data: bytes
    width: int
    height: int
    components: int
    bits_per_component: int
    format: int
    is_mask: bool
    jbig2_globals: Optional[bytes] = None

    @property
    def format_name(self):
        return image_format_name(self.format)


def image_format_name(fmt):
    return load_library().uphip_pdf_image_format_name(fmt).decode()


def is_pdf_file(filename):
    return bool(load_library().uphip_pdf_is_pdf_file(filename.encode() if filename else None))


def _meta_struct(meta):
    if meta is None:
        return None, ()
    m = A.PdfMetadata()
    keep = []
    for k in META_FIELDS:
        v = meta.get(k) if isinstance(meta, dict) else getattr(meta, k, None)
        if v is not None:
            b = v.encode()
            keep.append(b)
            setattr(m, k, b)
    return m, keep


class PdfDocument:
    def __init__(self, handle, keep=None):
        self.handle = handle
        self._keep = keep

    @classmethod
    def open(cls, path):
        L = load_library()
        h = L.uphip_pdf_open(path.encode())
        if not h:
            _fail(L, "pdf_open failed")
        return cls(h)

    @classmethod
    def open_memory(cls, data: bytes):
        L = load_library()
        buf = C.create_string_buffer(bytes(data), len(data))
        h = L.uphip_pdf_open_memory(buf, len(data))
        if not h:
            _fail(L, "pdf_open_memory failed")
        return cls(h, buf)

    def close(self):
        if self.handle:
            load_library().uphip_pdf_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def page_count(self):
        return load_library().uphip_pdf_page_count(self.handle)

    @property
    def needs_password(self):
        return bool(load_library().uphip_pdf_needs_password(self.handle))

    def page_info(self, page):
        L = load_library()
        info = A.PdfPageInfo()
        if L.uphip_pdf_get_page_info(self.handle, page, C.byref(info)) != 0:
            _fail(L, "pdf_get_page_info failed")
        return info.width, info.height, info.rotation

    def extract_page_image(self, page) -> PdfImage:
        L = load_library()
        im = A.PdfImage()
        if L.uphip_pdf_extract_page_image(self.handle, page, C.byref(im)) != 0:
            _fail(L, "pdf_extract_page_image failed")
        try:
            g = C.string_at(im.jbig2_globals, im.jbig2_globals_size) if im.jbig2_globals_size else None
            return PdfImage(C.string_at(im.data, im.size), im.width, im.height, im.components,
                            im.bits_per_component, im.format, bool(im.is_mask), g)
        finally:
            L.uphip_pdf_free_image(C.byref(im))

    def metadata(self):
        L = load_library()
        m = A.PdfMetadata()
        if L.uphip_pdf_get_metadata(self.handle, C.byref(m)) != 0:
            _fail(L, "pdf_get_metadata failed")
        try:
            return {k: (getattr(m, k).decode() if getattr(m, k) is not None else None)
                    for k in META_FIELDS}
        finally:
            L.uphip_pdf_free_metadata(C.byref(m))

    def page_probe(self, page, dpi=0):
        L = load_library()
        info = A.PnmInfo()
        if L.uphip_pdf_page_probe(self.handle, page, dpi, C.byref(info)) != 0:
            _fail(L, "pdf_page_probe failed")
        return info.width, info.height, info.format

    def read_page(self, page, dpi=0) -> HostImage:
        L = load_library()
        w, h, fmt = self.page_probe(page, dpi)
        img = HostImage(w, h, fmt)
        info = A.PnmInfo(w, h, fmt)
        if L.uphip_pdf_read_page(self.handle, page, dpi, img.data.ctypes.data, img.linesize,
                                 C.byref(info)) != 0:
            _fail(L, "pdf_read_page failed")
        return img


class PdfWriter:
    def __init__(self, handle, keep=()):
        self.handle = handle
        self._keep = keep

    @classmethod
    def create(cls, path, meta=None, dpi=0):
        L = load_library()
        m, keep = _meta_struct(meta)
        h = L.uphip_pdf_writer_create(path.encode(), C.byref(m) if m is not None else None, dpi)
        if not h:
            _fail(L, "pdf_writer_create failed")
        return cls(h, (m, keep))

    def _call(self, rc, what):
        if rc != 0:
            _fail(load_library(), what)

    def add_page_jpeg(self, data: bytes, width, height, dpi=0):
        self._call(load_library().uphip_pdf_writer_add_page_jpeg(self.handle, data, len(data), width,
                                                                 height, dpi), "add_page_jpeg failed")

    def add_page_jp2(self, data: bytes, width, height, dpi=0):
        self._call(load_library().uphip_pdf_writer_add_page_jp2(self.handle, data, len(data), width,
                                                                height, dpi), "add_page_jp2 failed")

    def add_page_pixels(self, pixels, width, height, stride, fmt, dpi=0):
        """pixels: a contiguous uint8 numpy array, rows `stride` bytes apart;
        fmt PIXEL_GRAY8 or PIXEL_RGB24."""
        self._call(load_library().uphip_pdf_writer_add_page_pixels(
            self.handle, pixels.ctypes.data, width, height, stride, fmt, dpi), "add_page_pixels failed")

    @property
    def page_count(self):
        return load_library().uphip_pdf_writer_page_count(self.handle)

    def close(self):
        h, self.handle = self.handle, None
        if h and load_library().uphip_pdf_writer_close(h) != 0:
            _fail(load_library(), "pdf_writer_close failed")

    def abort(self):
        h, self.handle = self.handle, None
        if h:
            load_library().uphip_pdf_writer_abort(h)

    def __del__(self):
        try:
            self.abort()
        except Exception:
            pass
