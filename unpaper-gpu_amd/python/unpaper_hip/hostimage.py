"""Host-side image container (AVFrame data[0]/linesize[0] peer) + PNM/PNG I/O.

Format mapping follows what the reference's FFmpeg decode yields for each
input (sheet_stages.c:75-122, file.c:96-124): 1-bit PNG/PBM -> MONOBLACK (PBM
P4 -> MONOWHITE), 8-bit gray -> GRAY8, gray+alpha -> Y400A, RGB -> RGB24,
palette -> RGB24 through the palette.
"""
import numpy as np

from .ctypes_abi import FMT_GRAY8, FMT_Y400A, FMT_RGB24, FMT_MONOWHITE, FMT_MONOBLACK

BYTES_PER_PIXEL = {FMT_GRAY8: 1, FMT_Y400A: 2, FMT_RGB24: 3}


def min_linesize(width, fmt):
    if fmt in BYTES_PER_PIXEL:
        return width * BYTES_PER_PIXEL[fmt]
    return (width + 7) // 8


class HostImage:
    """A frame in host memory: `data` is (height, linesize) uint8."""

    def __init__(self, width, height, fmt, data=None, background=(255, 255, 255),
                 abs_black_threshold=170):
        self.width = int(width)
        self.height = int(height)
        self.format = int(fmt)
        self.background = tuple(background)
        self.abs_black_threshold = int(abs_black_threshold)
        ls = (min_linesize(self.width, self.format) + 7) & ~7
        if data is None:
            data = np.zeros((self.height, ls), dtype=np.uint8)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if data.ndim != 2 or data.shape[0] != self.height or \
                data.shape[1] < min_linesize(self.width, self.format):
            raise ValueError("bad frame buffer shape %r" % (data.shape,))
        self.data = data

    @property
    def linesize(self):
        return self.data.shape[1]

    def copy(self):
        return HostImage(self.width, self.height, self.format, self.data.copy(),
                         self.background, self.abs_black_threshold)

    # -- packing helpers ---------------------------------------------------
    @classmethod
    def from_array(cls, arr, fmt, **kw):
        """arr: (H,W) gray / (H,W,3) rgb / (H,W,2) gray+alpha / (H,W) bool for mono
        (True = white)."""
        arr = np.asarray(arr)
        h, w = arr.shape[:2]
        img = cls(w, h, fmt, **kw)
        n = min_linesize(w, fmt)
        if fmt == FMT_GRAY8:
            img.data[:, :n] = arr.reshape(h, w)
        elif fmt == FMT_RGB24:
            img.data[:, :n] = arr.reshape(h, w * 3)
        elif fmt == FMT_Y400A:
            img.data[:, :n] = arr.reshape(h, w * 2)
        else:
            white = arr.astype(bool)
            bits = white if fmt == FMT_MONOBLACK else ~white
            img.data[:, :n] = np.packbits(bits, axis=1, bitorder="big")
        return img

    def to_rgb(self):
        """Expanded (H,W,3) uint8 view using get_pixel semantics (pixel.c:20-63)."""
        h, w = self.height, self.width
        n = min_linesize(w, self.format)
        raw = self.data[:, :n]
        if self.format == FMT_GRAY8:
            g = raw
            return np.repeat(g[:, :, None], 3, axis=2)
        if self.format == FMT_Y400A:
            g = raw.reshape(h, w, 2)[:, :, 0]
            return np.repeat(g[:, :, None], 3, axis=2)
        if self.format == FMT_RGB24:
            return raw.reshape(h, w, 3).copy()
        bits = np.unpackbits(raw, axis=1, bitorder="big")[:, :w].astype(bool)
        white = bits if self.format == FMT_MONOBLACK else ~bits
        g = np.where(white, 255, 0).astype(np.uint8)
        return np.repeat(g[:, :, None], 3, axis=2)

    def to_gray(self):
        rgb = self.to_rgb().astype(np.uint16)
        return ((rgb[:, :, 0] + rgb[:, :, 1] + rgb[:, :, 2]) // 3).astype(np.uint8)

    def payload(self):
        """Bytes of the visible pixels only (no row padding)."""
        return self.data[:, :min_linesize(self.width, self.format)]

    # -- file I/O ----------------------------------------------------------
    @classmethod
    def from_pil(cls, pil, **kw):
        mode = pil.mode
        if mode == "1":
            return cls.from_array(np.array(pil, dtype=bool), FMT_MONOBLACK, **kw)
        if mode == "L":
            return cls.from_array(np.array(pil), FMT_GRAY8, **kw)
        if mode == "LA":
            return cls.from_array(np.array(pil), FMT_Y400A, **kw)
        if mode == "RGB":
            return cls.from_array(np.array(pil), FMT_RGB24, **kw)
        if mode in ("P", "RGBA"):
            return cls.from_array(np.array(pil.convert("RGB")), FMT_RGB24, **kw)
        raise ValueError("unsupported PIL mode " + mode)

    @classmethod
    def load(cls, path, **kw):
        from PIL import Image
        with Image.open(path) as im:
            im.load()
            return cls.from_pil(im, **kw)

    def to_pil(self):
        from PIL import Image
        if self.format in (FMT_MONOWHITE, FMT_MONOBLACK):
            return Image.fromarray(self.to_gray() >= 128).convert("1")
        if self.format in (FMT_GRAY8, FMT_Y400A):
            return Image.fromarray(self.to_gray(), "L")
        return Image.fromarray(self.to_rgb(), "RGB")

    def save_pnm(self, path):
        """saveImageDirect (file.c:133-176): P5 / P6 / P4 (MONOWHITE)."""
        w, h = self.width, self.height
        with open(path, "wb") as f:
            if self.format == FMT_GRAY8:
                f.write(b"P5\n%d %d\n255\n" % (w, h))
            elif self.format == FMT_RGB24:
                f.write(b"P6\n%d %d\n255\n" % (w, h))
            elif self.format == FMT_MONOWHITE:
                f.write(b"P4\n%d %d\n" % (w, h))
            else:
                raise ValueError("save_pnm: convert to GRAY8/RGB24/MONOWHITE first")
            f.write(np.ascontiguousarray(self.payload()).tobytes())


def binarized_diff_ratio(golden_gray, result_gray, threshold=128):
    """compare_images (tests/unpaper_tests.py:26-53): L-convert, binarize at
    128, ratio of differing pixels."""
    if golden_gray.shape != result_gray.shape:
        return float("inf")
    a = golden_gray >= threshold
    b = result_gray >= threshold
    return float(np.count_nonzero(a != b)) / a.size
