"""Generates tests/golden/pdf/*.pdf and expected.json: PDF files covering the
container features the reader handles (csrc/pdf.cpp), written here by a
small independent writer (not the code under test), plus PIL-written files.

The reference's own samples (tests/pdf_samples in the reference: test_jpeg.pdf,
test_2page.pdf, test_jbig2.pdf, benchmark_jbig2_50page.pdf) are copied
alongside as data fixtures; their expectations come from the reference's
pdf_reader_test.c (page counts, a JPEG image on test_jpeg.pdf page 0) and
from an independent parse with PIL.PdfParser (tests/test_pdf.py).

expected.json holds, per file: page count, per page the image format,
width, height, components, bits per component, the sha256 of the extracted
bytes and, for pixel pages, the sha256 of the decoded rows (zlib / PIL).

Run: python tests/golden/make_pdf_fixtures.py  (deterministic)
"""
import hashlib
import io
import json
import os
import zlib

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "pdf")


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


class Doc:
    """Objects as bytes; serialised with a classic table or an xref stream,
    optionally packing non-stream objects into an object stream."""

    def __init__(self):
        self.objs = {}  # num -> (dict_bytes, stream_bytes or None)

    def add(self, num, body, stream=None):
        self.objs[num] = (body, stream)

    def serialise(self, xref_stream=False, objstm=False, header=b"%PDF-1.7\n%\xe2\xe3\xcf\xd3\n",
                  root=1, info=None, base=b"", prev=None, extra_trailer=b""):
        out = bytearray(base + (header if not base else b""))
        offsets = {}
        packed = []
        if objstm:
            packed = sorted(n for n, (b, s) in self.objs.items() if s is None)
        for num in sorted(self.objs):
            if num in packed:
                continue
            body, stream = self.objs[num]
            offsets[num] = len(out)
            out += b"%d 0 obj\n" % num
            if stream is None:
                out += body + b"\nendobj\n"
            else:
                out += body + b"\nstream\n" + stream + b"\nendstream\nendobj\n"
        size = max(self.objs) + 1
        compressed = {}
        if packed:
            stm_num = size
            size += 1
            head, data = [], bytearray()
            for k, num in enumerate(packed):
                head.append(b"%d %d" % (num, len(data)))
                data += self.objs[num][0] + b"\n"
                compressed[num] = (stm_num, k)
            head = b" ".join(head) + b"\n"
            z = zlib.compress(bytes(head + data))
            offsets[stm_num] = len(out)
            out += (b"%d 0 obj\n<< /Type /ObjStm /N %d /First %d /Filter /FlateDecode /Length %d >>\nstream\n"
                    % (stm_num, len(packed), len(head), len(z))) + z + b"\nendstream\nendobj\n"
        trailer_extra = b" /Root %d 0 R" % root + (b" /Info %d 0 R" % info if info else b"") + \
            (b" /Prev %d" % prev if prev is not None else b"") + extra_trailer
        if not xref_stream:
            xref_at = len(out)
            nums = sorted(offsets)
            out += b"xref\n"
            if base:  # an update: one subsection per object
                for num in nums:
                    out += b"%d 1\n%010d 00000 n\r\n" % (num, offsets[num])
            else:
                out += b"0 %d\n0000000000 65535 f\r\n" % size
                for num in range(1, size):
                    if num in offsets:
                        out += b"%010d 00000 n\r\n" % offsets[num]
                    else:
                        out += b"0000000000 65535 f\r\n"
            out += b"trailer\n<< /Size %d%s >>\nstartxref\n%d\n%%%%EOF\n" % (size, trailer_extra, xref_at)
            return bytes(out)
        xnum = size
        size += 1
        rows = bytearray()
        for num in range(size):
            if num in offsets:
                rows += bytes([1]) + offsets[num].to_bytes(4, "big") + b"\x00"
            elif num in compressed:
                s, k = compressed[num]
                rows += bytes([2]) + s.to_bytes(4, "big") + bytes([k])
            elif num == xnum:
                rows += bytes([1]) + len(out).to_bytes(4, "big") + b"\x00"
            else:
                rows += b"\x00" * 6
        # PNG Up predictor on the rows, as many writers emit
        cols = 6
        pred = bytearray()
        prevrow = bytes(cols)
        for r in range(0, len(rows), cols):
            row = rows[r:r + cols]
            pred += b"\x02" + bytes((row[i] - prevrow[i]) & 255 for i in range(cols))
            prevrow = row
        z = zlib.compress(bytes(pred))
        xref_at = len(out)
        out += (b"%d 0 obj\n<< /Type /XRef /Size %d /W [1 4 1] /Filter /FlateDecode "
                b"/DecodeParms << /Predictor 12 /Columns 6 >>%s /Length %d >>\nstream\n"
                % (xnum, size, trailer_extra, len(z))) + z + b"\nendstream\nendobj\n"
        out += b"startxref\n%d\n%%%%EOF\n" % xref_at
        return bytes(out)


def page_objs(doc, first, img_dict, img_bytes, w_pt, h_pt, parent=2, extra_page=b""):
    im, ct, pg = first, first + 1, first + 2
    doc.add(im, img_dict, img_bytes)
    content = b"q %g 0 0 %g 0 0 cm /Im0 Do Q" % (w_pt, h_pt)
    doc.add(ct, b"<< /Length %d >>" % len(content), content)
    doc.add(pg, b"<< /Type /Page /Parent %d 0 R /MediaBox [0 0 %g %g] /Resources << /XObject << /Im0 %d 0 R >> >>"
            b" /Contents %d 0 R%s >>" % (parent, w_pt, h_pt, im, ct, extra_page))
    return pg


def gradient(w, h, c):
    y, x = np.mgrid[0:h, 0:w]
    if c == 1:
        return ((x * 7 + y * 3) % 256).astype(np.uint8)
    return np.stack([(x * 5) % 256, (y * 9) % 256, (x + y) % 256], -1).astype(np.uint8)


def jpeg_bytes(arr, **kw):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", quality=90, **kw)
    return b.getvalue()


# ---------------------------------------------------------------------------
# JBIG2 generic-region encoder (T.88 6.2 with the E.2 MQ encoder), written
# from the standard for these fixtures: templates 0-3, typical prediction,
# adaptive template pixels; the decoder under test must give the bitmaps back
# ---------------------------------------------------------------------------
QE = [(0x5601, 1, 1, 1), (0x3401, 2, 6, 0), (0x1801, 3, 9, 0), (0x0AC1, 4, 12, 0), (0x0521, 5, 29, 0),
      (0x0221, 38, 33, 0), (0x5601, 7, 6, 1), (0x5401, 8, 14, 0), (0x4801, 9, 14, 0), (0x3801, 10, 14, 0),
      (0x3001, 11, 17, 0), (0x2401, 12, 18, 0), (0x1C01, 13, 20, 0), (0x1601, 29, 21, 0), (0x5601, 15, 14, 1),
      (0x5401, 16, 14, 0), (0x5101, 17, 15, 0), (0x4801, 18, 16, 0), (0x3801, 19, 17, 0), (0x3401, 20, 18, 0),
      (0x3001, 21, 19, 0), (0x2801, 22, 19, 0), (0x2401, 23, 20, 0), (0x2201, 24, 21, 0), (0x1C01, 25, 22, 0),
      (0x1801, 26, 23, 0), (0x1601, 27, 24, 0), (0x1401, 28, 25, 0), (0x1201, 29, 26, 0), (0x1101, 30, 27, 0),
      (0x0AC1, 31, 28, 0), (0x09C1, 32, 29, 0), (0x08A1, 33, 30, 0), (0x0521, 34, 31, 0), (0x0441, 35, 32, 0),
      (0x02A1, 36, 33, 0), (0x0221, 37, 34, 0), (0x0141, 38, 35, 0), (0x0111, 39, 36, 0), (0x0085, 40, 37, 0),
      (0x0049, 41, 38, 0), (0x0025, 42, 39, 0), (0x0015, 43, 40, 0), (0x0009, 44, 41, 0), (0x0005, 45, 42, 0),
      (0x0001, 45, 43, 0), (0x5601, 46, 46, 0)]


class MqEnc:
    def __init__(self):
        self.a, self.c, self.ct, self.b = 0x8000, 0, 12, None
        self.out = bytearray()
        self.idx, self.mps = {}, {}

    def _byteout(self):
        if self.b == 0xFF:
            self._emit(self.c >> 20, 0xFFFFF, 7)
        elif self.c < 0x8000000:
            self._emit(self.c >> 19, 0x7FFFF, 8)
        else:
            self.b += 1
            if self.b == 0xFF:
                self.c &= 0x7FFFFFF
                self._emit(self.c >> 20, 0xFFFFF, 7)
            else:
                self._emit(self.c >> 19, 0x7FFFF, 8)

    def _emit(self, byte, mask, ct):
        if self.b is not None:
            self.out.append(self.b)
        self.b = byte & 0xFF
        self.c &= mask
        self.ct = ct

    def _renorm(self):
        while True:
            self.a = (self.a << 1) & 0xFFFFFFFF
            self.c = (self.c << 1) & 0xFFFFFFFF
            self.ct -= 1
            if self.ct == 0:
                self._byteout()
            if self.a & 0x8000:
                break

    def encode(self, cx, d):
        i, m = self.idx.get(cx, 0), self.mps.get(cx, 0)
        qe, nmps, nlps, sw = QE[i]
        self.a -= qe
        if d == m:
            if self.a & 0x8000:
                self.c += qe
                return
            if self.a < qe:
                self.a = qe
            else:
                self.c += qe
            self.idx[cx] = nmps
        else:
            if self.a < qe:
                self.c += qe
            else:
                self.a = qe
            if sw:
                self.mps[cx] = 1 - m
            self.idx[cx] = nlps
        self._renorm()

    def flush(self):
        tempc = self.c + self.a
        self.c |= 0xFFFF
        if self.c >= tempc:
            self.c -= 0x8000
        self.c = (self.c << self.ct) & 0xFFFFFFFF
        self._byteout()
        self.c = (self.c << self.ct) & 0xFFFFFFFF
        self._byteout()
        if self.b != 0xFF:
            self.out.append(self.b)
        self.out += b"\xff\xac"
        return bytes(self.out)


def jbig2_context(bm, x, y, tmpl, at):
    def p(dx, dy):
        xx, yy = x + dx, y + dy
        return int(bm[yy, xx]) if 0 <= xx < bm.shape[1] and 0 <= yy < bm.shape[0] else 0
    if tmpl == 0:
        bits = [(-1, 0), (-2, 0), (-3, 0), (-4, 0), (at[0], at[1]), (2, -1), (1, -1), (0, -1), (-1, -1), (-2, -1),
                (at[2], at[3]), (at[4], at[5]), (1, -2), (0, -2), (-1, -2), (at[6], at[7])]
    elif tmpl == 1:
        bits = [(-1, 0), (-2, 0), (-3, 0), (at[0], at[1]), (2, -1), (1, -1), (0, -1), (-1, -1), (-2, -1),
                (2, -2), (1, -2), (0, -2), (-1, -2)]
    elif tmpl == 2:
        bits = [(-1, 0), (-2, 0), (at[0], at[1]), (1, -1), (0, -1), (-1, -1), (-2, -1), (1, -2), (0, -2), (-1, -2)]
    else:
        bits = [(-1, 0), (-2, 0), (-3, 0), (-4, 0), (at[0], at[1]), (1, -1), (0, -1), (-1, -1), (-2, -1), (-3, -1)]
    return sum(p(dx, dy) << k for k, (dx, dy) in enumerate(bits))


def jbig2_generic(bm, tmpl, tpgdon, at):
    enc = MqEnc()
    sltp = [0x9B25, 0x0795, 0x00E5, 0x0195][tmpl]
    ltp = 0
    h, w = bm.shape
    for y in range(h):
        if tpgdon:
            same = bool((bm[y] == (bm[y - 1] if y else 0)).all())
            enc.encode(sltp, int(same != bool(ltp)))
            ltp = int(same)
            if same:
                continue
        for x in range(w):
            enc.encode(jbig2_context(bm, x, y, tmpl, at), int(bm[y, x]))
    return enc.flush()


def jbig2_stream(bm, tmpl, tpgdon, at, striped=False, unknown_len=False):
    h, w = bm.shape

    def seg(num, typ, data, length=None):
        return (num.to_bytes(4, "big") + bytes([typ]) + b"\x00" + b"\x01" +
                (len(data) if length is None else length).to_bytes(4, "big") + data)
    page = (w.to_bytes(4, "big") + (0xFFFFFFFF if striped else h).to_bytes(4, "big") + bytes(8) + b"\x00" +
            ((0x8000 | h) if striped else 0).to_bytes(2, "big"))
    nat = 8 if tmpl == 0 else 2
    gflags = (tmpl << 1) | (8 if tpgdon else 0)
    data = jbig2_generic(bm, tmpl, tpgdon, at)
    region = (w.to_bytes(4, "big") + h.to_bytes(4, "big") + bytes(8) + b"\x00" + bytes([gflags]) +
              bytes(v & 255 for v in at[:nat]) + data)
    out = seg(0, 48, page)
    if unknown_len:
        out += seg(1, 38, region + h.to_bytes(4, "big"), 0xFFFFFFFF)
    else:
        out += seg(1, 38, region)
    if striped:
        out += seg(2, 50, (h - 1).to_bytes(4, "big"))
    out += seg(3, 49, b"")
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    expected = {}

    def record(name, data, pages):
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(data)
        expected[name] = {"pages": pages}

    def px_sha(arr):
        return sha(np.ascontiguousarray(arr).tobytes())

    # 1. xref stream + object stream: a Flate gray page (PNG predictor 15)
    #    and a DCT RGB page, the page tree nested two levels
    g = gradient(64, 48, 1)
    rgb = gradient(40, 30, 3)
    rows = b"".join(b"\x02" + ((g[r].astype(int) - (g[r - 1].astype(int) if r else 0)) & 255)
                    .astype(np.uint8).tobytes() for r in range(48))
    flate_pred = zlib.compress(rows)
    jrgb = jpeg_bytes(rgb)
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    d.add(2, b"<< /Type /Pages /Kids [3 0 R] /Count 2 /Resources << >> >>")
    d.add(3, b"<< /Type /Pages /Parent 2 0 R /Kids [6 0 R 9 0 R] /Count 2 /MediaBox [0 0 64 48] /Rotate 90 >>")
    page_objs(d, 4, b"<< /Type /XObject /Subtype /Image /Width 64 /Height 48 /ColorSpace /DeviceGray "
              b"/BitsPerComponent 8 /Filter /FlateDecode /DecodeParms << /Predictor 15 /Colors 1 /Columns 64 >> "
              b"/Length %d >>" % len(flate_pred), flate_pred, 64, 48, parent=3)
    page_objs(d, 7, b"<< /Type /XObject /Subtype /Image /Width 40 /Height 30 /ColorSpace /DeviceRGB "
              b"/BitsPerComponent 8 /Filter /DCTDecode /Length %d >>" % len(jrgb), jrgb, 40, 30, parent=3)
    d.objs[9] = (d.objs[9][0].replace(b"/MediaBox [0 0 40 30]", b"/MediaBox [0 0 40 30] /Rotate 0"), None)
    d.add(10, b"<< /Title (xref \\(stream\\)) /Author <FEFF00C9006C00E8> >>")
    record("xrefstream_objstm.pdf", d.serialise(xref_stream=True, objstm=True, info=10), [
        {"format": "FLATE", "w": 64, "h": 48, "c": 1, "bpc": 8, "data": sha(flate_pred), "pixels": px_sha(g),
         "box": [48, 64, 0]},
        {"format": "JPEG", "w": 40, "h": 30, "c": 3, "bpc": 8, "data": sha(jrgb), "box": [40, 30, 0]},
    ])
    expected["xrefstream_objstm.pdf"]["meta"] = {"title": "xref (stream)", "author": "Élè"}

    # 2. incremental update: page 1's image replaced by an appended revision;
    #    the page has two images (the larger one wins, pdf_reader.c:311-333)
    small = gradient(8, 8, 1)
    big = gradient(32, 24, 1)
    zs, zb = zlib.compress(small.tobytes()), zlib.compress(big.tobytes())
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    d.add(2, b"<< /Type /Pages /Kids [3 0 R] /Count 1 >>")
    d.add(3, b"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 32 24] /Resources << /XObject << /Ia 4 0 R /Ib 5 0 R >> >> >>")
    d.add(4, b"<< /Type /XObject /Subtype /Image /Width 8 /Height 8 /ColorSpace /DeviceGray /BitsPerComponent 8 "
          b"/Filter /FlateDecode /Length %d >>" % len(zs), zs)
    d.add(5, b"<< /Type /XObject /Subtype /Image /Width 16 /Height 16 /ColorSpace /DeviceGray /BitsPerComponent 8 "
          b"/Length 256 >>", bytes(256))
    base = d.serialise()
    startxref = int(base.rsplit(b"startxref", 1)[1].split()[0])
    u = Doc()
    u.add(5, b"<< /Type /XObject /Subtype /Image /Width 32 /Height 24 /ColorSpace /DeviceGray /BitsPerComponent 8 "
          b"/Filter /FlateDecode /Length 6 0 R >>", zb)
    u.add(6, b"%d" % len(zb))
    record("incremental.pdf", u.serialise(base=base, prev=startxref), [
        {"format": "FLATE", "w": 32, "h": 24, "c": 1, "bpc": 8, "data": sha(zb), "pixels": px_sha(big),
         "box": [32, 24, 0]},
    ])

    # 3. a damaged cross-reference: every offset 7 bytes off, startxref wrong
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    d.add(2, b"<< /Type /Pages /Kids [5 0 R] /Count 1 >>")
    page_objs(d, 3, b"<< /Type /XObject /Subtype /Image /Width 40 /Height 30 /ColorSpace /DeviceRGB "
              b"/BitsPerComponent 8 /Filter /DCTDecode /Length 999999 >>", jrgb, 40, 30)
    raw = d.serialise()
    head, tail = raw.rsplit(b"xref\n", 1)
    lines = tail.split(b"\r\n")
    fixed = [(b"%010d%s" % (int(l[:10]) + 7, l[10:]) if l[:10].isdigit() and l.endswith(b" n") else l) for l in lines]
    broken = head + b"xref\n" + b"\r\n".join(fixed)
    broken = broken.rsplit(b"startxref\n", 1)[0] + b"startxref\n12345678\n%%EOF\n"
    record("damaged_xref.pdf", broken, [
        {"format": "JPEG", "w": 40, "h": 30, "c": 3, "bpc": 8, "data": sha(jrgb), "box": [40, 30, 0]},
    ])

    # 4. filter chains and colour spaces: ASCII85 over Flate (RGB), LZW (gray),
    #    a 1-bit image with /Decode [1 0], an ICCBased gray JPEG with the
    #    CropBox smaller than the MediaBox, an indexed image (no pixel path)
    import base64
    rgb2 = gradient(24, 16, 3)
    a85 = base64.a85encode(zlib.compress(rgb2.tobytes())) + b"~>"
    gl = gradient(20, 10, 1)

    def lzw_encode(data):
        # a plain LZW encoder (EarlyChange 1), 9..12-bit codes
        dic = {bytes([i]): i for i in range(256)}
        nxt, width, out, acc, nbits = 258, 9, bytearray(), 0, 0

        def emit(code):
            nonlocal acc, nbits
            acc = (acc << width) | code
            nbits += width
            while nbits >= 8:
                out.append((acc >> (nbits - 8)) & 255)
                nbits -= 8
        emit(256)
        w = b""
        for c in data:
            wc = w + bytes([c])
            if wc in dic:
                w = wc
                continue
            emit(dic[w])
            if nxt < 4096:
                dic[wc] = nxt
                nxt += 1
                if nxt + 1 > (1 << width) and width < 12:
                    width += 1
            w = bytes([c])
        if w:
            emit(dic[w])
        emit(257)
        if nbits:
            out.append((acc << (8 - nbits)) & 255)
        return bytes(out)
    lz = lzw_encode(gl.tobytes())
    bits = np.zeros((12, 16), np.uint8)
    bits[::2, ::3] = 1
    packed1 = np.packbits(bits, axis=1)
    jg = jpeg_bytes(gradient(30, 20, 1))
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    d.add(2, b"<< /Type /Pages /Kids [5 0 R 8 0 R 11 0 R 14 0 R 17 0 R 21 0 R] /Count 6 >>")
    page_objs(d, 3, b"<< /Type /XObject /Subtype /Image /Width 24 /Height 16 /ColorSpace /DeviceRGB "
              b"/BitsPerComponent 8 /Filter [/ASCII85Decode /FlateDecode] /Length %d >>" % len(a85), a85, 24, 16)
    page_objs(d, 6, b"<< /Type /XObject /Subtype /Image /Width 20 /Height 10 /ColorSpace /DeviceGray "
              b"/BitsPerComponent 8 /Filter /LZWDecode /Length %d >>" % len(lz), lz, 20, 10)
    page_objs(d, 9, b"<< /Type /XObject /Subtype /Image /Width 16 /Height 12 /ColorSpace /DeviceGray "
              b"/BitsPerComponent 1 /Decode [1 0] /Length %d >>" % packed1.size, packed1.tobytes(), 16, 12)
    page_objs(d, 12, b"<< /Type /XObject /Subtype /Image /Width 30 /Height 20 /ColorSpace [/ICCBased 18 0 R] "
              b"/BitsPerComponent 8 /Filter /DCT /Length %d >>" % len(jg), jg, 30, 20,
              extra_page=b" /CropBox [5 5 25 15]")
    page_objs(d, 15, b"<< /Type /XObject /Subtype /Image /Width 4 /Height 4 /ColorSpace [/Indexed /DeviceRGB 1 <000000FFFFFF>] "
              b"/BitsPerComponent 8 /Length 16 >>", bytes(16), 4, 4)
    d.add(18, b"<< /N 1 /Length 4 >>", b"\x00\x00\x00\x00")
    page_objs(d, 19, b"<< /Type /XObject /Subtype /Image /Width 5 /Height 3 /ColorSpace /DeviceCMYK "
              b"/BitsPerComponent 8 /Length 60 >>", bytes(60), 5, 3)
    record("filters.pdf", d.serialise(), [
        {"format": "FLATE", "w": 24, "h": 16, "c": 3, "bpc": 8, "data": sha(zlib.compress(rgb2.tobytes())),
         "pixels": px_sha(rgb2), "box": [24, 16, 0]},
        {"format": "RAW", "w": 20, "h": 10, "c": 1, "bpc": 8, "data": sha(gl.tobytes()), "pixels": px_sha(gl),
         "box": [20, 10, 0]},
        {"format": "RAW", "w": 16, "h": 12, "c": 1, "bpc": 1, "data": sha(packed1.tobytes()),
         "pixels": px_sha(packed1), "pixfmt": "MONOWHITE", "box": [16, 12, 0]},
        {"format": "JPEG", "w": 30, "h": 20, "c": 1, "bpc": 8, "data": sha(jg), "box": [20, 10, 0]},
        {"format": "RAW", "w": 4, "h": 4, "c": 1, "bpc": 8, "data": sha(bytes(16)),
         "pixels": px_sha(np.zeros((4, 12), np.uint8)), "pixfmt": "RGB24", "box": [4, 4, 0]},
        {"format": "RAW", "w": 5, "h": 3, "c": 4, "bpc": 8, "data": sha(bytes(60)), "nopixels": True,
         "box": [5, 3, 0]},
    ])

    # 5. an encrypted trailer (refused: no decryption)
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    d.add(2, b"<< /Type /Pages /Kids [] /Count 0 >>")
    d.add(3, b"<< /Filter /Standard /V 1 /R 2 /O <00> /U <00> /P -4 >>")
    record("encrypted.pdf", d.serialise(extra_trailer=b" /Encrypt 3 0 R"), [])
    expected["encrypted.pdf"]["encrypted"] = True

    # 6. PIL's own writer: three JPEG pages (L, RGB, L) at 150 dpi
    ims = [Image.fromarray(gradient(48, 64, 1)), Image.fromarray(gradient(36, 24, 3)),
           Image.fromarray(gradient(48, 64, 1))]
    b = io.BytesIO()
    ims[0].save(b, "PDF", resolution=150.0, save_all=True, append_images=ims[1:])
    pages = []
    for im in ims:
        c = 1 if im.mode == "L" else 3
        pages.append({"format": "JPEG", "w": im.width, "h": im.height, "c": c, "bpc": 8,
                      "box": [round(im.width * 72 / 150, 3), round(im.height * 72 / 150, 3), 0]})
    record("pil_multipage.pdf", b.getvalue(), pages)

    # 7. a JPEG 2000 page (JPXDecode) from the codec fixtures
    with open(os.path.join(HERE, "j2k", "gray.jp2"), "rb") as f:
        jp2 = f.read()
    gw, gh = Image.open(io.BytesIO(jp2)).size
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    d.add(2, b"<< /Type /Pages /Kids [5 0 R] /Count 1 >>")
    page_objs(d, 3, b"<< /Type /XObject /Subtype /Image /Width %d /Height %d /Filter /JPXDecode /Length %d >>"
              % (gw, gh, len(jp2)), jp2, gw, gh)
    record("jpx.pdf", d.serialise(), [
        {"format": "JPEG2000", "w": gw, "h": gh, "c": 1, "bpc": 8, "data": sha(jp2), "box": [gw, gh, 0]},
    ])

    # 8. JBIG2 generic regions: templates 0 (moved AT pixels) to 3, typical
    #    prediction, a striped page with an end-of-stripe and an unknown-length
    #    region; expanded to GRAY8 as jbig2_expand_to_gray8 (1 -> 0, 0 -> 255)
    rng = np.random.default_rng(88)
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    cases = [(0, False, [2, -1, -4, -1, 1, -2, -3, -2], {}), (1, True, [3, -1], {}), (2, False, [2, -1], {}),
             (3, True, [2, -1], {"striped": True, "unknown_len": True}), (0, True, [3, -1, -3, -1, 2, -2, -2, -2], {})]
    kids, pages = [], []
    for k, (tmpl, tp, at, kw) in enumerate(cases):
        h, w = 37 + 3 * k, 61 + 5 * k
        bm = np.zeros((h, w), np.uint8)
        for _ in range(12):  # blobs and lines, repeated rows for typical prediction
            y0, x0 = rng.integers(0, h - 6), rng.integers(0, w - 10)
            bm[y0:y0 + rng.integers(1, 6), x0:x0 + rng.integers(2, 10)] = 1
        bm[h // 2:h // 2 + 4] = bm[h // 2]
        stream = jbig2_stream(bm, tmpl, tp, at, **kw)
        first = 3 + 3 * k
        kids.append(b"%d 0 R" % (first + 2))
        page_objs(d, first, b"<< /Type /XObject /Subtype /Image /Width %d /Height %d /ColorSpace /DeviceGray "
                  b"/BitsPerComponent 1 /Filter /JBIG2Decode /Length %d >>" % (w, h, len(stream)), stream, w, h)
        pages.append({"format": "JBIG2", "w": w, "h": h, "c": 1, "bpc": 1, "data": sha(stream),
                      "pixels": px_sha(np.where(bm == 1, 0, 255).astype(np.uint8)), "pixfmt": "GRAY8",
                      "box": [w, h, 0]})
    d.add(2, b"<< /Type /Pages /Kids [%s] /Count %d >>" % (b" ".join(kids), len(kids)))
    record("jbig2_generic.pdf", d.serialise(), pages)

    # 9. CCITT fax pages: PIL's own bilevel PDF (Group 4, /BlackIs1 true), and
    #    libtiff's Group 3 strips (1-D, 2-D, with EOL fill bits) wrapped with
    #    the matching /DecodeParms; one page with /BlackIs1 false and
    #    /Decode [1 0] (the two inversions cancel).  Expected pixels: PIL's
    #    image, white 255 / black 0.
    from PIL import ImageDraw

    def bilevel(w, h, seed):
        r = np.random.default_rng(seed)
        im = Image.new("1", (w, h), 1)
        dr = ImageDraw.Draw(im)
        for _ in range(30):
            x0, y0 = int(r.integers(0, w)), int(r.integers(0, h))
            dr.rectangle([x0, y0, x0 + int(r.integers(0, w // 3 + 1)), y0 + int(r.integers(0, 6))], fill=0)
        for _ in range(12):
            dr.text((int(r.integers(0, w)), int(r.integers(0, h))), "Scan 42", fill=0)
        return im

    def gray_of(im):
        return np.where(np.asarray(im), 255, 0).astype(np.uint8)
    ims = [bilevel(201, 90, 1), bilevel(2600, 40, 2)]  # the second needs the extended make-up codes
    b = io.BytesIO()
    ims[0].save(b, "PDF", save_all=True, append_images=ims[1:])
    record("ccitt_pil.pdf", b.getvalue(), [
        {"format": "CCITT", "w": im.width, "h": im.height, "c": 1, "bpc": 1, "pixels": px_sha(gray_of(im)),
         "pixfmt": "GRAY8", "box": [im.width, im.height, 0]} for im in ims])
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    kids, pages = [], []
    for k, (opts, black1) in enumerate([(0, True), (1, True), (4, True), (5, True), (1, False)]):
        im = bilevel(300, 60 + k, 10 + k)
        t = io.BytesIO()
        im.save(t, "TIFF", compression="group3", tiffinfo={278: im.height, 292: opts})
        tg = Image.open(io.BytesIO(t.getvalue())).tag_v2
        strip = t.getvalue()[tg[273][0]:tg[273][0] + tg[279][0]]
        parms = b"<< /K %d /Columns %d /Rows %d /BlackIs1 %s%s >>" % (
            opts & 1, im.width, im.height, b"true" if black1 else b"false",
            b" /EncodedByteAlign true /EndOfLine true" if opts & 4 else b"")
        first = 3 + 3 * k
        kids.append(b"%d 0 R" % (first + 2))
        page_objs(d, first, b"<< /Type /XObject /Subtype /Image /Width %d /Height %d /ColorSpace /DeviceGray "
                  b"/BitsPerComponent 1 /Filter /CCITTFaxDecode /DecodeParms %s%s /Length %d >>"
                  % (im.width, im.height, parms, b"" if black1 else b" /Decode [1 0]", len(strip)),
                  strip, im.width, im.height)
        pages.append({"format": "CCITT", "w": im.width, "h": im.height, "c": 1, "bpc": 1, "data": sha(strip),
                      "pixels": px_sha(gray_of(im)), "pixfmt": "GRAY8", "box": [im.width, im.height, 0]})
    d.add(2, b"<< /Type /Pages /Kids [%s] /Count %d >>" % (b" ".join(kids), len(kids)))
    record("ccitt_g3.pdf", d.serialise(), pages)

    # 10. palette images: PIL's own (ASCIIHex, /Indexed /DeviceRGB 255 with a
    #     hex-string lookup) and a 4-bit index stream with a gray base and a
    #     stream lookup; expected: PIL's RGB conversion / the lookup applied
    r = np.random.default_rng(9)
    a = r.integers(0, 200, (30, 41)).astype(np.uint8)
    pim = Image.fromarray(a, "P")
    pim.putpalette(list(r.integers(0, 256, 768).astype(np.uint8)))
    b = io.BytesIO()
    pim.save(b, "PDF")
    record("palette_pil.pdf", b.getvalue(), [
        {"format": "RAW", "w": 41, "h": 30, "c": 1, "bpc": 8, "pixels": px_sha(np.asarray(pim.convert("RGB"))),
         "pixfmt": "RGB24", "box": [41, 30, 0]}])
    idx = r.integers(0, 16, (7, 9)).astype(np.uint8)
    packed4 = np.zeros((7, 5), np.uint8)
    for x in range(9):
        packed4[:, x // 2] |= idx[:, x] << (4 if x % 2 == 0 else 0)
    lut = r.integers(0, 256, 16).astype(np.uint8)
    d = Doc()
    d.add(1, b"<< /Type /Catalog /Pages 2 0 R >>")
    d.add(2, b"<< /Type /Pages /Kids [5 0 R] /Count 1 >>")
    z4 = zlib.compress(packed4.tobytes())
    page_objs(d, 3, b"<< /Type /XObject /Subtype /Image /Width 9 /Height 7 /ColorSpace [/Indexed /DeviceGray 15 6 0 R] "
              b"/BitsPerComponent 4 /Filter /FlateDecode /Length %d >>" % len(z4), z4, 9, 7)
    d.add(6, b"<< /Length 16 >>", lut.tobytes())
    record("palette_4bit.pdf", d.serialise(), [
        {"format": "FLATE", "w": 9, "h": 7, "c": 1, "bpc": 4, "data": sha(z4), "pixels": px_sha(lut[idx]),
         "pixfmt": "GRAY8", "box": [9, 7, 0]}])

    with open(os.path.join(OUT, "expected.json"), "w") as f:
        json.dump(expected, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
