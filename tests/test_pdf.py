"""The PDF container (csrc/pdf.cpp; include/unpaper_hip.h "PDF container"):
the reference's pdf/pdf_reader.h, pdf/pdf_writer.h and the PDF pipeline
(pdf/pdf_pipeline_cpu_batch.c) without MuPDF.

Oracles:
  * the reference's own samples (tests/pdf_samples there, copied to
    tests/golden/pdf) with what its pdf_reader_test.c / pdf_writer_test.c
    expect (page counts, a JPEG on test_jpeg.pdf, metadata, Producer);
  * an independent parse of the same files with PIL.PdfParser (classic
    cross-reference files) and zlib for Flate pixels;
  * tests/golden/make_pdf_fixtures.py: files written by a separate Python
    writer covering xref streams, object streams, incremental updates, a
    damaged xref, filter chains and colour spaces, with expected.json;
  * GPU: pages through the runner equal the oracle on the decoded pages,
    and the PDF sink's pages equal the JPEG / JPEG 2000 sinks' files.
"""
import ctypes as C
import hashlib
import io
import json
import os
import zlib

import numpy as np
import pytest
from PIL import Image, PdfParser

from unpaper_hip import ctypes_abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "pdf")
EXPECTED = json.load(open(os.path.join(FIX, "expected.json")))
FMT_BYTES = {A.FMT_GRAY8: 1, A.FMT_RGB24: 3}


def _pdf():
    from unpaper_hip import pdf
    return pdf


def _err():
    from unpaper_hip.device import load_library
    L = load_library()
    e = L.uphip_last_error()
    L.uphip_clear_error()
    return e.decode() if e else ""


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def rows(img):
    n = img.width * FMT_BYTES[img.format] if img.format in FMT_BYTES else (img.width + 7) // 8
    return np.ascontiguousarray(img.data[:, :n])


def pil_images(path):
    """page -> (width, height, filter names, raw stream bytes) of the page's
    largest image, through PIL's parser (independent of csrc/pdf.cpp)."""
    with open(path, "rb") as f:
        p = PdfParser.PdfParser(f=f)
        out = []
        for pg in p.pages:
            page = p.read_indirect(pg)
            res = page[b"Resources"]
            if isinstance(res, PdfParser.IndirectReference):
                res = p.read_indirect(res)
            xo = res[b"XObject"]
            best = None
            for _, ref in xo.items():
                s = p.read_indirect(ref)
                d = s.dictionary
                area = d[b"Width"] * d[b"Height"]
                if best is None or area > best[0]:
                    flt = d.get(b"Filter")
                    flt = [] if flt is None else [flt] if not isinstance(flt, list) else flt
                    best = (area, d[b"Width"], d[b"Height"], [bytes(x) for x in flt], bytes(s.buf))
            out.append(best[1:])
        p.close()
        return out


def regex_images(path):
    """The same as pil_images for flat files PIL's parser refuses (indirect
    /Length): objects found by a regular expression, stream lengths from
    /Length (direct or an integer object), the pages' /XObject references
    followed -- a second, independent reading for the reference's samples."""
    import re
    data = open(path, "rb").read()
    heads = {int(m.group(1)): m.end() for m in re.finditer(rb"(?<![0-9])(\d+) 0 obj", data)}

    def body(num):
        at = heads[num]
        m = re.compile(rb"\s*(<<.*?>>)\s*(stream\r?\n|endobj)", re.S).match(data, at)
        if not m:  # a bare value
            return re.compile(rb"\s*(.*?)\s*endobj", re.S).match(data, at).group(1), None
        d = m.group(1)
        if not m.group(2).startswith(b"stream"):
            return d, None
        ln = re.search(rb"/Length (\d+)( 0 R)?", d)
        n = int(body(int(ln.group(1)))[0]) if ln.group(2) else int(ln.group(1))
        return d, data[m.end():m.end() + n]

    pages = []
    for num in sorted(heads):
        d, _ = body(num)
        if re.search(rb"/Type\s*/Page(?![s])", d):
            pages.append(d)
    out = []
    kids = re.search(rb"/Kids\s*\[([^]]*)\]", body(int(re.search(rb"/Pages (\d+) 0 R", data).group(1)))[0])
    order = [int(k) for k in re.findall(rb"(\d+) 0 R", kids.group(1))]
    for pnum in order:
        d = body(pnum)[0]
        xo = re.search(rb"/XObject\s*<<(.*?)>>", d, re.S).group(1)
        best = None
        for ref in re.findall(rb"/\w+\s+(\d+) 0 R", xo):
            idict, stream = body(int(ref))
            w = int(re.search(rb"/Width (\d+)", idict).group(1))
            h = int(re.search(rb"/Height (\d+)", idict).group(1))
            flt = re.findall(rb"/(\w+Decode)", idict)
            if best is None or w * h > best[0]:
                best = (w * h, w, h, flt, stream)
        out.append(best[1:])
    return out


# ---------------------------------------------------------------------------
# reader (host; no GPU)
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_reader_fixtures(name):
    pdf = _pdf()
    e = EXPECTED[name]
    d = pdf.PdfDocument.open(os.path.join(FIX, name))
    assert d.needs_password == bool(e.get("encrypted"))
    if e.get("encrypted"):
        with pytest.raises(Exception, match="encrypted"):
            d.extract_page_image(0)
        return
    assert d.page_count == len(e["pages"])
    for i, p in enumerate(e["pages"]):
        im = d.extract_page_image(i)
        assert (im.format_name, im.width, im.height, im.components, im.bits_per_component) == \
            (p["format"], p["w"], p["h"], p["c"], p["bpc"]), (name, i)
        if "data" in p:
            assert sha(im.data) == p["data"], (name, i)
        w, h, rot = d.page_info(i)
        assert abs(w - p["box"][0]) < 1e-3 and abs(h - p["box"][1]) < 1e-3 and rot == p["box"][2], (name, i)
        if "pixels" in p:  # Flate / raw pages decode on the host
            img = d.read_page(i)
            assert sha(rows(img)) == p["pixels"], (name, i)
            if "pixfmt" in p:
                assert img.format == getattr(A, "FMT_" + p["pixfmt"])
        if p.get("nopixels"):
            with pytest.raises(Exception, match="not supported"):
                d.read_page(i)
    if "meta" in e:
        m = d.metadata()
        for k, v in e["meta"].items():
            assert m[k] == v


def test_reference_samples():
    """pdf_reader_test.c: test_jpeg.pdf has one page with an extractable
    JPEG, test_2page.pdf two pages; the JBIG2 files' pages are JBIG2 images
    (no decoder here: refused with the cause)."""
    pdf = _pdf()
    d = pdf.PdfDocument.open(os.path.join(FIX, "test_jpeg.pdf"))
    assert d.page_count == 1
    w, h, rot = d.page_info(0)
    assert w > 0 and h > 0 and rot == 0
    im = d.extract_page_image(0)
    assert im.format_name == "JPEG" and (im.width, im.height) == (2480, 3507) and im.components == 1
    assert im.data[:3] == b"\xff\xd8\xff"
    m = d.metadata()
    assert m["title"] == "test_jpeg" and m["producer"] == "https://imagemagick.org"
    assert m["creation_date"].startswith("D:2025")
    d2 = pdf.PdfDocument.open(os.path.join(FIX, "test_2page.pdf"))
    assert d2.page_count == 2
    assert [d2.page_info(i)[:2] for i in range(2)] == [(2480.0, 3507.0), (1240.0, 1754.0)]
    for name, n in (("test_jbig2.pdf", 1), ("benchmark_jbig2_50page.pdf", 50)):
        d3 = pdf.PdfDocument.open(os.path.join(FIX, name))
        assert d3.page_count == n
        im = d3.extract_page_image(n - 1)
        assert im.format_name == "JBIG2" and im.bits_per_component == 1 and im.components == 1


# sha256 of the GRAY8 expansion of the reference's JBIG2 samples (csrc/jbig2.cpp;
# the generic-region pages decode to clean documents -- a wrong context
# template turns arithmetic decoding into noise at once -- and equal the
# per-pixel form below; the text-region page is a symbol instance)
JBIG2_PAGES = {
    ("benchmark_jbig2_50page.pdf", 0): "017b9cf4bf2a5a38c7dc9806f8c15b017fd65a2d200bab4cb99a834aa332feee",
    ("benchmark_jbig2_50page.pdf", 49): "e6de7561b233e4bd7fdc31191d76aeda100975c16bc071642cd53512b9eea2e4",
    ("test_jbig2.pdf", 0): "442cc982f9820c5e8042008121425760dd6fa85739a10f737b1f2928db28ef6b",
}


def test_jbig2_reference_samples():
    """jbig2_decode_test.c: test_jbig2.pdf's page is 200x100 with both black
    and white pixels (here: a black 81x61 symbol at (20, 20)); the 50-page
    benchmark (jbig2 -p generic regions, template 0) decodes page by page;
    1 = black expands to GRAY8 0 (lib/jbig2_decode.c:136-170)."""
    pdf = _pdf()
    for (name, page), digest in JBIG2_PAGES.items():
        d = pdf.PdfDocument.open(os.path.join(FIX, name))
        assert d.page_probe(page, 0) == (d.extract_page_image(page).width, d.extract_page_image(page).height,
                                         A.FMT_GRAY8)
        img = d.read_page(page)
        a = rows(img)
        assert set(np.unique(a)) <= {0, 255} and (a == 0).any() and (a == 255).any()
        assert sha(a) == digest, (name, page)
    d = pdf.PdfDocument.open(os.path.join(FIX, "test_jbig2.pdf"))
    a = rows(d.read_page(0))
    ys, xs = np.nonzero(a == 0)
    assert (ys.min(), ys.max(), xs.min(), xs.max()) == (20, 80, 20, 100)
    # the benchmark at the reference's PDF dpi (300) passes the page-size check
    d = pdf.PdfDocument.open(os.path.join(FIX, "benchmark_jbig2_50page.pdf"))
    assert d.page_probe(3, 300) == (2480, 3508, A.FMT_GRAY8)


def test_jbig2_fast_path_equals_per_pixel():
    """Template 0 with the nominal AT pixels runs on sliding context windows;
    UPH_JBIG2_GENERIC=1 forces the per-pixel context: same pages."""
    import subprocess
    import sys
    code = ("import sys, hashlib, numpy as np; sys.path.insert(0, %r)\n"
            "from unpaper_hip import pdf\n"
            "d = pdf.PdfDocument.open(%r)\n"
            "print(hashlib.sha256(np.ascontiguousarray(d.read_page(0).data[:, :2480]).tobytes()).hexdigest())\n"
            % (os.path.join(ROOT, "unpaper-gpu_amd", "python"), os.path.join(FIX, "benchmark_jbig2_50page.pdf")))
    env = dict(os.environ, UPH_JBIG2_GENERIC="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == JBIG2_PAGES[("benchmark_jbig2_50page.pdf", 0)]


def test_jbig2_refusals():
    """Segments outside the decoder's scope fail with their name."""
    pdf = _pdf()
    data = open(os.path.join(FIX, "jbig2_generic.pdf"), "rb").read()
    d = pdf.PdfDocument.open_memory(data)
    im = d.extract_page_image(0)
    stream = im.data
    # MMR bit on the generic region flags (segment 1's data byte 17)
    seg1 = 11 + 19
    mmr = bytearray(stream)
    mmr[seg1 + 11 + 17] |= 1
    # a halftone region segment type
    half = bytearray(stream)
    half[seg1 + 4] = 22
    for bad, what in ((mmr, "MMR"), (half, "halftone")):
        fixed = data.replace(stream, bytes(bad))
        with pytest.raises(Exception, match=what):
            pdf.PdfDocument.open_memory(fixed).read_page(0)


@pytest.mark.parametrize("name", ["test_jpeg.pdf", "test_2page.pdf", "pil_multipage.pdf", "filters.pdf",
                                  "incremental.pdf", "jpx.pdf", "test_jbig2.pdf", "ccitt_pil.pdf"])
def test_reader_matches_independent_parse(name):
    """The largest image of every page equals what PIL's parser finds: the
    raw bytes of DCT / JPX / JBIG2 / Flate streams; Flate pixels equal
    zlib's inflate of PIL's stream bytes."""
    pdf = _pdf()
    path = os.path.join(FIX, name)
    try:
        ref = pil_images(path)
    except PdfParser.PdfFormatError:  # indirect /Length: the regular-expression reading
        ref = regex_images(path)
    d = pdf.PdfDocument.open(path)
    assert d.page_count == len(ref)
    for i, (w, h, flt, raw) in enumerate(ref):
        im = d.extract_page_image(i)
        assert (im.width, im.height) == (w, h)
        last = flt[-1] if flt else None
        if last in (b"DCTDecode", b"JPXDecode", b"JBIG2Decode", b"FlateDecode", b"CCITTFaxDecode") and len(flt) == 1:
            assert im.data == raw, (name, i)
        if last == b"FlateDecode" and len(flt) == 1 and im.bits_per_component == 8:
            px = np.frombuffer(zlib.decompress(raw), np.uint8)
            got = rows(d.read_page(i)).reshape(-1)
            assert (got == px[:got.size]).all() and got.size == px.size, (name, i)


def test_reference_2page_pixels_match_zlib():
    """test_2page.pdf's Flate pages decode on the host to zlib's inflate of
    the streams (PIL's parser for the bytes)."""
    pdf = _pdf()
    path = os.path.join(FIX, "test_2page.pdf")
    d = pdf.PdfDocument.open(path)
    for i, (w, h, _, raw) in enumerate(regex_images(path)):
        img = d.read_page(i)
        assert img.format == A.FMT_GRAY8 and (img.width, img.height) == (w, h)
        assert (rows(img).reshape(-1) == np.frombuffer(zlib.decompress(raw), np.uint8)).all()


def test_reader_dpi_check():
    """pdf_pipeline_decode.c:69-111: with a dpi, an image more than 4 px off
    the page size at that dpi would be rendered by the reference -- refused
    here; dpi 0 takes the image."""
    pdf = _pdf()
    d = pdf.PdfDocument.open(os.path.join(FIX, "test_2page.pdf"))
    assert d.page_probe(0, 72) == (2480, 3507, A.FMT_GRAY8)  # 2480 pt at 72 dpi
    assert d.page_probe(0, 0) == (2480, 3507, A.FMT_GRAY8)
    with pytest.raises(Exception, match="rendering"):
        d.page_probe(0, 300)
    d = pdf.PdfDocument.open(os.path.join(FIX, "pil_multipage.pdf"))
    assert d.page_probe(0, 150) == (48, 64, A.FMT_GRAY8)
    assert d.page_probe(1, 152) == (36, 24, A.FMT_RGB24)  # within 4 px
    with pytest.raises(Exception, match="rendering"):
        d.page_probe(0, 300)


def test_reader_errors():
    pdf = _pdf()
    with pytest.raises(Exception):
        pdf.PdfDocument.open(os.path.join(FIX, "missing.pdf"))
    with pytest.raises(Exception, match="PDF"):
        pdf.PdfDocument.open_memory(b"not a pdf at all, just text" * 4)
    d = pdf.PdfDocument.open(os.path.join(FIX, "filters.pdf"))
    for bad in (-1, 6, 1 << 20):
        with pytest.raises(Exception, match="out of range"):
            d.extract_page_image(bad)
        with pytest.raises(Exception, match="out of range"):
            d.page_info(bad)
    # a page without images (e.g. vector content) names rendering
    data = open(os.path.join(FIX, "incremental.pdf"), "rb").read()
    nov = data.replace(b"/XObject << /Ia 4 0 R /Ib 5 0 R >>", b"/Font << /Ia 4 0 R /Ib 5 0 R >>   ")
    assert len(nov) == len(data)
    with pytest.raises(Exception, match="rendering"):
        pdf.PdfDocument.open_memory(nov).extract_page_image(0)
    from unpaper_hip.device import load_library
    L = load_library()
    assert L.uphip_pdf_page_count(None) == -1
    assert L.uphip_pdf_get_page_info(None, 0, None) == -1
    assert _err()
    L.uphip_pdf_close(None)
    L.uphip_pdf_free_image(None)
    assert pdf.is_pdf_file("a.PDF") and pdf.is_pdf_file("/x/y.pdf") and not pdf.is_pdf_file("a.png")
    # a PDF handed to the single-image readers names the document path
    info = A.PnmInfo()
    assert L.uphip_image_probe(os.path.join(FIX, "filters.pdf").encode(), C.byref(info)) == -1
    assert "uphip_source_pdf" in _err()
    assert not pdf.is_pdf_file(None)
    assert [pdf.image_format_name(k) for k in range(9)] == [
        "UNKNOWN", "JPEG", "JPEG2000", "JBIG2", "CCITT", "PNG", "RAW", "FLATE", "UNKNOWN"]


@pytest.mark.parametrize("name", ["xrefstream_objstm.pdf", "incremental.pdf", "filters.pdf", "damaged_xref.pdf",
                                  "test_2page.pdf"])
def test_reader_survives_damage(name):
    """Truncations and byte flips: every call returns (an error or a
    result), none crashes (the same cases run under ASan in
    tests/c/sanitize_main.c)."""
    pdf = _pdf()
    data = open(os.path.join(FIX, name), "rb").read()
    rng = np.random.default_rng(len(data))
    cases = [data[:k] for k in (10, 100, len(data) // 3, len(data) // 2, len(data) - 40, len(data) - 5)]
    for _ in range(24):
        b = bytearray(data)
        for q in rng.integers(0, len(b), 8):
            b[q] = int(rng.integers(0, 256))
        cases.append(bytes(b))
    for c in cases:
        try:
            d = pdf.PdfDocument.open_memory(c)
        except Exception:
            continue
        for i in range(min(d.page_count, 3)):
            for f in (d.page_info, d.extract_page_image, d.metadata):
                try:
                    f(i) if f != d.metadata else f()
                except Exception:
                    pass
            try:
                im = d.extract_page_image(i)
                if im.format_name in ("FLATE", "RAW"):
                    d.read_page(i)
            except Exception:
                pass
    _err()


# ---------------------------------------------------------------------------
# writer (host; no GPU)
# ---------------------------------------------------------------------------

def jpeg_bytes(arr, q=90):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", quality=q)
    return b.getvalue()


def test_writer_round_trip(tmp_path):
    """pdf_writer_test.c: JPEG, JP2 and pixel pages, metadata preserved,
    Producer "unpaper", page sizes from the dpi; read back by our reader and
    by PIL's parser."""
    pdf = _pdf()
    rng = np.random.default_rng(5)
    g = rng.integers(0, 256, (40, 30), dtype=np.uint8)
    rgb = rng.integers(0, 256, (20, 50, 3), dtype=np.uint8)
    jg, jc = jpeg_bytes(g), jpeg_bytes(rgb)
    jp2 = open(os.path.join(ROOT, "tests", "golden", "j2k", "rgb_mct.jp2"), "rb").read()
    jw, jh = Image.open(io.BytesIO(jp2)).size
    path = str(tmp_path / "out.pdf")
    meta = {"title": "Test PDF Title", "author": "Test Author", "subject": "Grüße ☃",
            "creation_date": "D:20250101000000Z"}
    w = pdf.PdfWriter.create(path, meta, 150)
    w.add_page_jpeg(jg, 30, 40)
    w.add_page_jpeg(jc, 50, 20, dpi=72)
    w.add_page_jp2(jp2, jw, jh)
    pix = np.zeros((40, 32), np.uint8)
    pix[:, :30] = g
    w.add_page_pixels(pix, 30, 40, 32, pdf.PIXEL_GRAY8)
    w.add_page_pixels(np.ascontiguousarray(rgb), 50, 20, 150, pdf.PIXEL_RGB24)
    assert w.page_count == 5
    assert not os.path.exists(path)  # streamed to path.part until close
    w.close()
    assert os.path.exists(path) and not os.path.exists(path + ".part")
    d = pdf.PdfDocument.open(path)
    assert d.page_count == 5
    m = d.metadata()
    assert m["title"] == "Test PDF Title" and m["author"] == "Test Author"
    assert m["subject"] == "Grüße ☃" and m["producer"] == "unpaper"
    assert m["creation_date"] == "D:20250101000000Z" and m["keywords"] is None
    sizes = [(30 * 72 / 150, 40 * 72 / 150), (50.0, 20.0), (jw * 72 / 150, jh * 72 / 150),
             (30 * 72 / 150, 40 * 72 / 150), (50 * 72 / 150, 20 * 72 / 150)]
    for i, (pw, ph) in enumerate(sizes):
        bw, bh, rot = d.page_info(i)
        assert abs(bw - pw) < 1e-3 and abs(bh - ph) < 1e-3 and rot == 0, i
    im = [d.extract_page_image(i) for i in range(5)]
    assert [x.format_name for x in im] == ["JPEG", "JPEG", "JPEG2000", "FLATE", "FLATE"]
    assert im[0].data == jg and im[1].data == jc and im[2].data == jp2
    assert [x.components for x in im] == [1, 3, 3, 1, 3]
    assert (rows(d.read_page(3)) == g).all()
    assert (rows(d.read_page(4)).reshape(20, 50, 3) == rgb).all()
    # PIL's parser agrees
    ref = pil_images(path)
    assert [r[:2] for r in ref] == [(30, 40), (50, 20), (jw, jh), (30, 40), (50, 20)]
    assert ref[0][3] == jg and ref[2][3] == jp2
    assert np.frombuffer(zlib.decompress(ref[4][3]), np.uint8).tobytes() == rgb.tobytes()
    with open(path, "rb") as f:
        p = PdfParser.PdfParser(f=f)
        info = p.info
        assert info[b"Producer"] == b"unpaper" and info[b"Title"] == b"Test PDF Title"
        p.close()


def test_writer_abort_and_errors(tmp_path):
    pdf = _pdf()
    path = str(tmp_path / "aborted.pdf")
    w = pdf.PdfWriter.create(path)
    w.add_page_jpeg(jpeg_bytes(np.zeros((8, 8), np.uint8)), 8, 8)
    w.abort()
    assert not os.path.exists(path) and not os.path.exists(path + ".part")
    w = pdf.PdfWriter.create(str(tmp_path / "e.pdf"), None, 0)
    with pytest.raises(Exception, match="dimensions"):
        w.add_page_jpeg(b"\xff\xd8\xff", 0, 10)
    with pytest.raises(Exception, match="Invalid"):
        w.add_page_jpeg(b"", 10, 10)
    with pytest.raises(Exception, match="stride"):
        w.add_page_pixels(np.zeros(100, np.uint8), 10, 10, 5, pdf.PIXEL_RGB24)
    with pytest.raises(Exception, match="format"):
        w.add_page_pixels(np.zeros(100, np.uint8), 10, 10, 10, 7)
    assert w.page_count == 0
    w.close()  # an empty document is valid
    d = pdf.PdfDocument.open(str(tmp_path / "e.pdf"))
    assert d.page_count == 0
    from unpaper_hip.device import load_library
    L = load_library()
    assert not L.uphip_pdf_writer_create(None, None, 0)
    assert _err()
    assert not L.uphip_pdf_writer_create(str(tmp_path / "no" / "dir.pdf").encode(), None, 0)
    assert _err()
    assert L.uphip_pdf_writer_page_count(None) == 0
    assert L.uphip_pdf_writer_close(None) == 0
    L.uphip_pdf_writer_abort(None)


def test_sink_pdf_argument_checks(tmp_path):
    from unpaper_hip.device import load_library
    L = load_library()
    p = str(tmp_path / "s.pdf").encode()
    assert not L.uphip_sink_pdf(None, None, 0, 0, 0)
    assert not L.uphip_sink_pdf(p, None, 0, 0, 2)
    assert not L.uphip_sink_pdf(p, None, 0, 101, 0)
    assert not L.uphip_sink_pdf(p, None, 5000, 0, 0)
    assert _err()
    k = L.uphip_sink_pdf(p, None, 0, 0, 1)
    assert k
    L.uphip_sink_destroy(k)  # unfinished: no file
    assert not os.path.exists(p.decode()) and not os.path.exists(p.decode() + ".part")
    k = L.uphip_sink_pdf(p, None, 0, 0, 0)
    assert L.uphip_sink_finish(k) == 0 and L.uphip_sink_finish(k) == 0
    L.uphip_sink_destroy(k)
    assert os.path.exists(p.decode())
    assert not L.uphip_source_pdf(None, 0)
    assert "null path" in _err()
    assert not L.uphip_source_pdf(os.path.join(FIX, "encrypted.pdf").encode(), 0)
    assert "encrypted" in _err()
    s = L.uphip_source_pdf(os.path.join(FIX, "test_2page.pdf").encode(), 0)
    assert s and L.uphip_source_page_count(s) == 2
    L.uphip_source_destroy(s)


# ---------------------------------------------------------------------------
# GPU: device decode of PDF pages, the runner's PDF source and sink
# ---------------------------------------------------------------------------

def page_arr(w, h, seed, rgb=False):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    g = np.full((h, w), 255, np.uint8)
    for r in range(3, h - 6, 9):
        for c0 in range(2, w - 10, 13):
            if rng.random() < 0.6:
                g[r:r + 5, c0:c0 + rng.integers(2, 10)] = rng.integers(0, 70)
    g[: h // 5] = ((x * 3 + y * 7) % 256)[: h // 5]
    if not rgb:
        return g
    return np.stack([g, np.roll(g, 7, 1), np.maximum(g, 90)], 2)


@pytest.mark.gpu
def test_read_page_device_codecs(hip):
    """JPEG and JPEG 2000 pages decode on the device to PIL's pixels (the
    codecs' own parity: libjpeg islow / OpenJPEG)."""
    pdf = _pdf()
    for name, pages in (("test_jpeg.pdf", [0]), ("pil_multipage.pdf", [0, 1, 2]), ("jpx.pdf", [0]),
                        ("xrefstream_objstm.pdf", [1]), ("filters.pdf", [3]), ("damaged_xref.pdf", [0])):
        d = pdf.PdfDocument.open(os.path.join(FIX, name))
        for i in pages:
            img = d.read_page(i)
            ref = np.asarray(Image.open(io.BytesIO(d.extract_page_image(i).data)))
            got = rows(img)
            assert (got.reshape(ref.shape) == ref).all(), (name, i)


@pytest.mark.gpu
def test_runner_pdf_source_and_sinks(hip, oracle, tmp_path):
    """The PDF pipeline: a PDF whose pages are JPEG, Flate and JPEG 2000
    images of one geometry through uphip_source_pdf; the sheets equal the
    oracle on the decoded pages; the PDF sink's JPEG pages equal the JPEG
    sink's files and its JPEG 2000 pages the JP2 sink's (same run, same
    device encoders), in page order, with the input's metadata."""
    from unpaper_hip.hostimage import HostImage
    from unpaper_hip.pipeline import (Runner, sink_jp2, sink_jpeg, sink_pdf, sink_pnm, source_pdf,
                                      source_page_count, pnm_read)
    pdf = _pdf()
    w, h = 320, 400
    opts = oracle.default_options()
    src = str(tmp_path / "in.pdf")
    wr = pdf.PdfWriter.create(src, {"title": "scan", "author": "me"}, 100)
    decoded = []
    for i in range(5):
        a = page_arr(w, h, 70 + i)
        if i in (0, 3):
            j = jpeg_bytes(a, 85)
            wr.add_page_jpeg(j, w, h)
            decoded.append(np.asarray(Image.open(io.BytesIO(j))))
        elif i == 2:
            jp2_path = str(tmp_path / "p.jp2")
            Image.fromarray(a).save(jp2_path, "JPEG2000")
            j = open(jp2_path, "rb").read()
            wr.add_page_jp2(j, w, h)
            decoded.append(np.asarray(Image.open(io.BytesIO(j))))
        else:
            wr.add_page_pixels(np.ascontiguousarray(a), w, h, w, pdf.PIXEL_GRAY8)
            decoded.append(a)
    wr.close()
    exp = []
    for px in decoded:
        sheet, fmt, _ = oracle.process_sheet(opts, [HostImage.from_array(px, A.FMT_GRAY8)])
        exp.append(oracle.convert_for_save(sheet, fmt))
    s = source_pdf(src, 100)
    assert source_page_count(s) == 5
    r = Runner(opts, 2, w, h, A.FMT_GRAY8, devices=(0,), streams=2, host_threads=3)
    meta = pdf.PdfDocument.open(src).metadata()
    try:
        failed, err = r.run_host(5, s, sink_pnm(str(tmp_path / "o%02d.pgm")))
        assert failed == 0, err
        failed, err = r.run_host(5, s, sink_jpeg(str(tmp_path / "o%02d.jpg")))
        assert failed == 0, err
        failed, err = r.run_host(5, s, sink_jp2(str(tmp_path / "o%02d.jp2")))
        assert failed == 0, err
        outs = {}
        for mode in (0, 1):
            k = sink_pdf(str(tmp_path / ("out%d.pdf" % mode)), meta, 0, 0, mode)
            failed, err = r.run_host(5, s, k)
            assert failed == 0, err
            k.finish()
            outs[mode] = str(tmp_path / ("out%d.pdf" % mode))
    finally:
        r.close()
    for i in range(5):
        got = pnm_read(str(tmp_path / ("o%02d.pgm" % i)))
        assert (got.payload() == exp[i].payload()).all(), i
    for mode, ext, fmt in ((0, "jpg", "JPEG"), (1, "jp2", "JPEG2000")):
        d = pdf.PdfDocument.open(outs[mode])
        assert d.page_count == 5
        m = d.metadata()
        assert m["title"] == "scan" and m["author"] == "me" and m["producer"] == "unpaper"
        for i in range(5):
            im = d.extract_page_image(i)
            assert im.format_name == fmt
            assert im.data == open(tmp_path / ("o%02d.%s" % (i, ext)), "rb").read(), (mode, i)
            pw, ph, _ = d.page_info(i)
            assert abs(pw - w * 72 / 300) < 1e-3 and abs(ph - h * 72 / 300) < 1e-3
    # the lossless pages decode back to the sheets
    d = pdf.PdfDocument.open(outs[1])
    for i in range(5):
        assert (rows(d.read_page(i)) == pnm_read(str(tmp_path / ("o%02d.pgm" % i))).payload()).all()


@pytest.mark.gpu
def test_runner_host_decoded_pdf_pages(hip, oracle, tmp_path):
    """JBIG2 and CCITT pages (decoded on the runner's load pool by the PDF
    source) through the pipeline equal the oracle on the same decoded pages:
    jobs 0..page of the document (pages of one geometry), sheets to PGM."""
    from unpaper_hip.hostimage import HostImage
    from unpaper_hip.pipeline import Runner, sink_pnm, source_pdf, pnm_read
    pdf = _pdf()
    opts = oracle.default_options()
    for name, page in (("jbig2_generic.pdf", 0), ("ccitt_g3.pdf", 0), ("ccitt_pil.pdf", 0),
                       ("test_jbig2.pdf", 0), ("benchmark_jbig2_50page.pdf", 3)):
        path = os.path.join(FIX, name)
        d = pdf.PdfDocument.open(path)
        w, h, fmt = d.page_probe(page, 0)
        assert fmt == A.FMT_GRAY8 and all(d.page_probe(i, 0) == (w, h, fmt) for i in range(page + 1))
        px = rows(d.read_page(page))
        sheet, ofmt, _ = oracle.process_sheet(opts, [HostImage.from_array(px, A.FMT_GRAY8)])
        exp = oracle.convert_for_save(sheet, ofmt)
        out = str(tmp_path / ("o_%s_%%02d.pgm" % name.replace(".", "_")))
        r = Runner(opts, 2, w, h, A.FMT_GRAY8, devices=(0,), streams=2, host_threads=2)
        try:
            failed, err = r.run_host(page + 1, source_pdf(path, 0), sink_pnm(out))
        finally:
            r.close()
        assert failed == 0, err
        assert (pnm_read(out % page).payload() == exp.payload()).all(), (name, page)


# ---------------------------------------------------------------------------
# the reference's own PDF unit tests (tests/pdf_reader_test.c,
# tests/pdf_writer_test.c in the reference), compiled where they lie against
# integration/pdf_hip.c -- the reference's reader / writer API on this
# library instead of MuPDF (make adapter; built here, run here and on the box)
# ---------------------------------------------------------------------------
REF_PDF = {k: os.path.join(ROOT, "tests", "c", "_build", "ref_pdf_%s_test" % k) for k in ("reader", "writer")}
REF_PDF["jbig2"] = os.path.join(ROOT, "tests", "c", "_build", "ref_jbig2_decode_test")


def _ref_pdf_run(which, tmp_path):
    import subprocess
    exe = REF_PDF[which]
    if not os.path.exists(exe):
        if not os.path.isdir("/root/reference/tests"):
            pytest.skip("reference tree absent and %s not prebuilt" % exe)
        subprocess.check_call(["make", "-s", os.path.relpath(exe, ROOT)], cwd=ROOT)
    # the tests find tests/pdf_samples beside $TEST_IMGSRC_DIR and a JPEG in it
    (tmp_path / "source_images").mkdir()
    os.symlink(FIX, tmp_path / "pdf_samples")
    Image.fromarray((np.arange(120 * 90).reshape(90, 120) % 251).astype(np.uint8)).save(
        tmp_path / "source_images" / "test_jpeg.jpg", quality=90)
    env = dict(os.environ, TEST_IMGSRC_DIR=str(tmp_path / "source_images"))
    return subprocess.run([exe], cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)


def test_reference_pdf_writer_unit_tests(tmp_path):
    """The reference's pdf_writer_test.c passes unchanged on integration/pdf_hip.c."""
    r = _ref_pdf_run("writer", tmp_path)
    assert r.returncode == 0 and "All tests passed!" in r.stdout, r.stdout + r.stderr
    assert "FAILED" not in r.stdout and "SKIPPED" not in r.stdout


def test_reference_pdf_reader_unit_tests_host(tmp_path):
    """The reference's pdf_reader_test.c up to its render tests, which need
    the device JPEG decode (the GPU test below runs them)."""
    r = _ref_pdf_run("reader", tmp_path)
    out = r.stdout
    head = out.split("Test: pdf_render_page...")[0]
    assert head.count("PASSED") == 8 and "FAILED" not in head and "SKIPPED" not in head, out
    assert "(2480x3507, JPEG, 1444986 bytes)" in head


@pytest.mark.gpu
def test_reference_pdf_reader_unit_tests(hip, tmp_path):
    """All of pdf_reader_test.c, render tests included (image pages: the
    page's image decoded on the device, box-resampled to the page at 150 dpi)."""
    r = _ref_pdf_run("reader", tmp_path)
    assert r.returncode == 0 and "All tests passed!" in r.stdout, r.stdout + r.stderr
    assert "FAILED" not in r.stdout and "SKIPPED" not in r.stdout


def test_reference_jbig2_unit_tests(tmp_path):
    """The reference's jbig2_decode_test.c (built with JBIG2 and PDF on)
    passes unchanged on integration/jbig2_hip.c + pdf_hip.c: test_jbig2.pdf
    decodes to 200x100 with both colours after the gray expansion."""
    r = _ref_pdf_run("jbig2", tmp_path)
    assert r.returncode == 0 and "All tests passed!" in r.stdout, r.stdout + r.stderr
    assert r.stdout.count("PASSED") == 4 and "FAILED" not in r.stdout and "skipped" not in r.stdout
    assert "(200x100, stride=25)" in r.stdout
