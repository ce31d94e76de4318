/* sanitize_main.c — host code under AddressSanitizer + UndefinedBehavior-
 * Sanitizer: the oracle's whole sheet pipeline on synthetic
 * pages in every input format and layout, plus the product library's host
 * PNM codec (pnm.cpp) and PNG decoder (png.cpp) on well-formed and
 * malformed files.  No GPU involved.
 * Built and run by `make sanitize` (tests/test_sanitize.py).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/unpaper_hip.h"
#include "../../oracle/oracle.h"
#include "../../unpaper-gpu_amd/csrc/synth.h"

static int g_fail;

static OImage page(int fmt, int w, int h, uint32_t seed) {
  OImage im = o_create_image((UphipRectangleSize){w, h}, fmt, false, (UphipPixel){255, 255, 255},
                             170);
  for (int y = 0; y < h; y++) {
    uint8_t *row = im.data + (int64_t)y * im.linesize;
    if (fmt >= UPHIP_FMT_MONOWHITE) memset(row, 0, (size_t)im.linesize);
    for (int x = 0; x < w; x++) {
      const uint8_t v = synth_pixel(seed, w, h, x, y);
      if (fmt == UPHIP_FMT_GRAY8) row[x] = v;
      else if (fmt == UPHIP_FMT_Y400A) { row[2 * x] = v; row[2 * x + 1] = 255; }
      else if (fmt == UPHIP_FMT_RGB24) { row[3 * x] = v; row[3 * x + 1] = v / 2 + 100; row[3 * x + 2] = v; }
      else if ((v < 128) == (fmt == UPHIP_FMT_MONOWHITE)) row[x >> 3] |= (uint8_t)(0x80 >> (x & 7));
    }
  }
  return im;
}

static void sheet(const char *what, UphipOptions *o, int fmt, int w, int h, uint32_t seed) {
  OImage pages[2] = {page(fmt, w, h, seed), page(fmt, w, h, seed + 1)};
  OImage out;
  int32_t ofmt = 0;
  OReport rep;
  if (o_process_sheet(o, pages, &out, &ofmt, &rep) != 0) {
    fprintf(stderr, "process_sheet failed: %s\n", what);
    g_fail++;
  } else {
    OImage saved = o_convert_for_save(out, ofmt);
    o_free_image(&saved);
    o_free_image(&out);
  }
  o_free_image(&pages[0]);
  o_free_image(&pages[1]);
}

static void codec(const char *dir) {
  char path[512];
  snprintf(path, sizeof path, "%s/s.pgm", dir);
  uint8_t img[7 * 5];
  for (int i = 0; i < 35; i++) img[i] = (uint8_t)(i * 7);
  if (uphip_pnm_write(path, img, 7, 7, 5, UPHIP_FMT_GRAY8) != 0) g_fail++;
  uint8_t back[8 * 5];
  UphipPnmInfo info;
  if (uphip_pnm_probe(path, &info) != 0 || uphip_pnm_read(path, back, 8, &info) != 0) g_fail++;
  for (int y = 0; y < 5; y++)
    if (memcmp(back + 8 * y, img + 7 * y, 7)) g_fail++;
  static const char *bad[] = {"P5\n4 4\n255\n\x01", "P6 99999999999 1 255 ", "P2 2 2 255 1 2 x",
                              "P1 9 1 1 0 1", "P4\n16 2\n\xff", "P3 1 1 255", "#", "",
                              /* 2^31 does not fit int32_t; a raster past the size bound */
                              "P5 2147483648 1 255 ", "P5 2147483647 1 255 ",
                              "P6 1048576 1048576 255 "};
  for (size_t i = 0; i < sizeof bad / sizeof *bad; i++) {
    snprintf(path, sizeof path, "%s/b%zu.pnm", dir, i);
    FILE *f = fopen(path, "wb");
    fwrite(bad[i], 1, strlen(bad[i]), f);
    fclose(f);
    uint8_t buf[64];
    UphipPnmInfo want = {4, 4, UPHIP_FMT_GRAY8};
    if (uphip_pnm_probe(path, &info) == 0 && (info.width <= 0 || info.height <= 0)) {
      fprintf(stderr, "malformed file %zu probed as %dx%d\n", i, info.width, info.height);
      g_fail++;
    }
    if (uphip_pnm_read(path, buf, 16, &want) == 0) {
      fprintf(stderr, "malformed file %zu accepted\n", i);
      g_fail++;
    }
    uphip_clear_error();
  }
}

/* the PNG decoder (png.cpp) on the reference's own sources and on
 * truncated / bit-flipped copies of one */
static void png(const char *dir, const char *fixtures) {
  static const char *names[] = {"imgsrc002.png", "imgsrc003.png", "imgsrc004.png", "imgsrc006.png"};
  char path[512];
  for (size_t i = 0; i < sizeof names / sizeof *names; i++) {
    snprintf(path, sizeof path, "%s/%s", fixtures, names[i]);
    UphipPnmInfo info;
    if (uphip_image_probe(path, &info) != 0) {
      fprintf(stderr, "png probe %s: %s\n", path, uphip_last_error());
      g_fail++;
      continue;
    }
    const int64_t ls = info.format == UPHIP_FMT_RGB24 ? 3 * (int64_t)info.width
                       : info.format == UPHIP_FMT_MONOBLACK ? (info.width + 7) / 8
                                                            : (int64_t)info.width;
    uint8_t *buf = (uint8_t *)malloc((size_t)(ls * info.height));
    if (uphip_image_read(path, buf, ls, &info) != 0) g_fail++;
    if (i == 3) {  /* damaged copies of the small RGB source */
      FILE *f = fopen(path, "rb");
      static uint8_t raw[1 << 20];
      const size_t n = fread(raw, 1, sizeof raw, f);
      fclose(f);
      for (size_t cut = 9; cut < n; cut += n / 13) {
        for (int flip = 0; flip < 2; flip++) {
          snprintf(path, sizeof path, "%s/bad.png", dir);
          f = fopen(path, "wb");
          if (flip) {
            raw[cut] ^= 0x41;
            fwrite(raw, 1, n, f);
            raw[cut] ^= 0x41;
          } else {
            fwrite(raw, 1, cut, f);
          }
          fclose(f);
          if (!flip && uphip_image_read(path, buf, ls, &info) == 0) {
            fprintf(stderr, "truncated png (%zu bytes) accepted\n", cut);
            g_fail++;
          }
          if (flip) uphip_image_read(path, buf, ls, &info);  /* must not crash */
          uphip_clear_error();
        }
      }
    }
    free(buf);
  }
}

/* the JPEG host decoder (jpeg.cpp: markers + Huffman, sequential and
 * progressive) on small PIL-encoded files (tests/golden/jpeg), and truncated /
 * bit-flipped copies (truncated ones must fail, none may crash) */
static void jpeg(const char *fixtures) {
  static const char *good[] = {"gray.jpg", "rgb420_rst.jpg", "rgb444_opt.jpg", "progressive.jpg"};
  static uint8_t raw[1 << 16], tmp[1 << 16];
  char path[512];
  for (size_t i = 0; i < sizeof good / sizeof *good; i++) {
    const int refuse = 0;
    snprintf(path, sizeof path, "%s/../jpeg/%s", fixtures, good[i]);
    FILE *f = fopen(path, "rb");
    if (!f) {
      fprintf(stderr, "jpeg fixture %s missing\n", path);
      g_fail++;
      continue;
    }
    const size_t n = fread(raw, 1, sizeof raw, f);
    fclose(f);
    const int64_t need = uphip_jpeg_entropy_decode(raw, n, NULL, 0);
    if ((need < 0) != refuse) {
      fprintf(stderr, "jpeg %s: %s\n", path, need < 0 ? uphip_last_error() : "accepted");
      g_fail++;
    }
    uphip_clear_error();
    if (need > 0) {
      void *packed = malloc((size_t)need);
      if (uphip_jpeg_entropy_decode(raw, n, packed, need) != need) g_fail++;
      free(packed);
    }
    for (size_t cut = 3; cut < n; cut += n / 17 + 1) {
      /* cut inside the entropy-coded data (not the trailing EOI alone) */
      if (cut + 2 < n && uphip_jpeg_entropy_decode(raw, cut, NULL, 0) >= 0) {
        fprintf(stderr, "truncated jpeg %s (%zu of %zu bytes) accepted\n", path, cut, n);
        g_fail++;
      }
      uphip_clear_error();
      memcpy(tmp, raw, n);
      tmp[cut] ^= 0x5A;
      uphip_jpeg_entropy_decode(tmp, n, NULL, 0); /* must not crash */
      uphip_clear_error();
    }
  }
}

/* the JPEG 2000 host half (j2k.cpp: boxes, markers, packet headers, tag
 * trees, the MQ decoder and the coding passes) on the committed fixtures
 * (tests/golden/j2k) and cut / bit-flipped copies: the fixtures must decode,
 * nothing may crash */
static void j2k(const char *fixtures) {
  static const char *good[] = {"gray.jp2",         "rgb_mct.jp2",      "rgb_nomct.jp2",
                               "tiled_rpcl.j2k",   "offset_tiles.jp2", "lossy_layers.jp2",
                               "lossy_rgb.jp2",    "plt.jp2"};
  static uint8_t raw[1 << 16], tmp[1 << 16];
  char path[512];
  unsigned seed = 12345;
  for (size_t i = 0; i < sizeof good / sizeof *good; i++) {
    snprintf(path, sizeof path, "%s/../j2k/%s", fixtures, good[i]);
    FILE *f = fopen(path, "rb");
    if (!f) {
      fprintf(stderr, "j2k fixture %s missing\n", path);
      g_fail++;
      continue;
    }
    const size_t n = fread(raw, 1, sizeof raw, f);
    fclose(f);
    UphipPnmInfo info;
    const int64_t need = uphip_jp2_entropy_decode(raw, n, NULL, 0, &info);
    if (need <= 0) {
      fprintf(stderr, "j2k %s: %s\n", path, uphip_last_error());
      g_fail++;
    }
    uphip_clear_error();
    for (size_t cut = 0; cut < n; cut += n / 29 + 1) {
      uphip_jp2_entropy_decode(raw, cut, NULL, 0, &info); /* must not crash */
      uphip_clear_error();
      for (int k = 0; k < 3; k++) {
        memcpy(tmp, raw, n);
        seed = seed * 1103515245u + 12345u;
        tmp[(cut + (seed >> 8)) % n] ^= (uint8_t)(1 + (seed >> 24) % 255);
        uphip_jp2_entropy_decode(tmp, n, NULL, 0, &info);
        uphip_clear_error();
      }
    }
    /* crafted SIZ: huge tiles and offsets (XO = XTO = 10, XT = YT = INT_MAX;
     * then XT = 0x80000000, read as a negative int32): the tile bounds must
     * not overflow */
    for (size_t q = 0; q + 40 < n; q++) {
      if (raw[q] != 0xFF || raw[q + 1] != 0x51) continue;
      static const uint32_t xt[] = {0x7FFFFFFFu, 0x80000000u, 0xFFFFFFFFu};
      for (int v = 0; v < 3; v++) {
        memcpy(tmp, raw, n);
        uint8_t *z = tmp + q + 6; /* X, Y, XO, YO, XT, YT, XTO, YTO (big-endian u32) */
        const uint32_t vals[8] = {0, 0, 10, 10, xt[v], xt[v], 10, 10};
        for (int k = 2; k < 8; k++) {
          z[4 * k] = (uint8_t)(vals[k] >> 24);
          z[4 * k + 1] = (uint8_t)(vals[k] >> 16);
          z[4 * k + 2] = (uint8_t)(vals[k] >> 8);
          z[4 * k + 3] = (uint8_t)vals[k];
        }
        uphip_jp2_entropy_decode(tmp, n, NULL, 0, &info); /* fails or decodes; never UB */
        uphip_clear_error();
      }
      break;
    }
  }
}

/* the PDF reader on the fixtures (tests/golden/pdf), their truncations and
 * byte flips: open, page info, image extraction, host pixel decode and the
 * metadata must fail cleanly or succeed, never touch memory out of bounds;
 * then a writer round trip */
static void pdf_case(const UphipPdfDocument *unused, const uint8_t *p, size_t n) {
  (void)unused;
  UphipPdfDocument *d = uphip_pdf_open_memory(p, n);
  if (!d) {
    uphip_clear_error();
    return;
  }
  const int np = uphip_pdf_page_count(d);
  static uint8_t px[1 << 20];
  for (int i = 0; i < np && i < 6; i++) {
    UphipPdfPageInfo info;
    UphipPdfImage im;
    UphipPnmInfo g;
    uphip_pdf_get_page_info(d, i, &info);
    if (uphip_pdf_extract_page_image(d, i, &im) == 0) uphip_pdf_free_image(&im);
    if (uphip_pdf_page_probe(d, i, 0, &g) == 0 && (g.format == UPHIP_FMT_GRAY8 || g.format == UPHIP_FMT_RGB24 ||
                                                   g.format >= UPHIP_FMT_MONOWHITE)) {
      const int64_t ls = g.format == UPHIP_FMT_RGB24 ? 3 * (int64_t)g.width
                         : g.format == UPHIP_FMT_GRAY8 ? g.width : ((int64_t)g.width + 7) / 8;
      if (ls * g.height <= (int64_t)sizeof px) {
        UphipPdfImage im2;
        if (uphip_pdf_extract_page_image(d, i, &im2) == 0) {
          if (im2.format == UPHIP_PDF_IMAGE_FLATE || im2.format == UPHIP_PDF_IMAGE_RAW ||
              im2.format == UPHIP_PDF_IMAGE_JBIG2 || im2.format == UPHIP_PDF_IMAGE_CCITT)
            uphip_pdf_read_page(d, i, 0, px, ls, &g);
          uphip_pdf_free_image(&im2);
        }
      }
    }
    uphip_clear_error();
  }
  UphipPdfMetadata m;
  if (uphip_pdf_get_metadata(d, &m) == 0) uphip_pdf_free_metadata(&m);
  uphip_pdf_close(d);
  uphip_clear_error();
}

static void pdf(const char *dir, const char *fixtures) {
  static const char *good[] = {"xrefstream_objstm.pdf", "incremental.pdf", "damaged_xref.pdf", "filters.pdf",
                               "pil_multipage.pdf",     "jpx.pdf",         "encrypted.pdf",    "test_jbig2.pdf",
                               "jbig2_generic.pdf",     "ccitt_pil.pdf",   "ccitt_g3.pdf",
                               "palette_pil.pdf",       "palette_4bit.pdf"};
  static uint8_t raw[1 << 16], tmp[1 << 16];
  char path[512];
  unsigned seed = 777;
  for (size_t i = 0; i < sizeof good / sizeof *good; i++) {
    snprintf(path, sizeof path, "%s/../pdf/%s", fixtures, good[i]);
    FILE *f = fopen(path, "rb");
    if (!f) {
      fprintf(stderr, "pdf fixture %s missing\n", path);
      g_fail++;
      continue;
    }
    const size_t n = fread(raw, 1, sizeof raw, f);
    fclose(f);
    UphipPdfDocument *d = uphip_pdf_open_memory(raw, n);
    if (!d || (uphip_pdf_page_count(d) <= 0 && !uphip_pdf_needs_password(d))) {
      fprintf(stderr, "pdf %s: %s\n", path, uphip_last_error());
      g_fail++;
    }
    uphip_pdf_close(d);
    uphip_clear_error();
    pdf_case(NULL, raw, n);
    for (size_t cut = 1; cut < n; cut += n / 23 + 1) {
      pdf_case(NULL, raw, cut);
      for (int k = 0; k < 3; k++) {
        memcpy(tmp, raw, n);
        seed = seed * 1103515245u + 12345u;
        tmp[(cut + (seed >> 8)) % n] ^= (uint8_t)(1 + (seed >> 24) % 255);
        pdf_case(NULL, tmp, n);
      }
    }
  }
  snprintf(path, sizeof path, "%s/san.pdf", dir);
  UphipPdfMetadata meta = {0};
  meta.title = (char *)"t\xc3\xa9st (1)";
  UphipPdfWriter *w = uphip_pdf_writer_create(path, &meta, 200);
  static uint8_t g[33 * 17];
  for (size_t k = 0; k < sizeof g; k++) g[k] = (uint8_t)(k * 7);
  if (!w || uphip_pdf_writer_add_page_pixels(w, g, 30, 17, 33, 0, 0) != 0 ||
      uphip_pdf_writer_add_page_pixels(w, g, 11, 17, 33, 1, 0) != 0 || uphip_pdf_writer_close(w) != 0) {
    fprintf(stderr, "pdf writer: %s\n", uphip_last_error());
    g_fail++;
    return;
  }
  UphipPdfDocument *d = uphip_pdf_open(path);
  UphipPdfMetadata m;
  if (!d || uphip_pdf_page_count(d) != 2 || uphip_pdf_get_metadata(d, &m) != 0 || !m.title ||
      strcmp(m.title, meta.title) != 0) {
    fprintf(stderr, "pdf writer round trip: %s\n", uphip_last_error());
    g_fail++;
  } else {
    uphip_pdf_free_metadata(&m);
  }
  uphip_pdf_close(d);
  remove(path);
}

/* crafted JPEG headers: an over-subscribed Huffman table must
 * be refused before it indexes the lookahead table, and a frame claiming far
 * more blocks than the file holds must fail without sizing anything from it */
static size_t put16(uint8_t *p, size_t i, int v) {
  p[i] = (uint8_t)(v >> 8);
  p[i + 1] = (uint8_t)v;
  return i + 2;
}

static void jpeg_crafted(void) {
  static uint8_t f[4096];
  for (int variant = 0; variant < 3; variant++) {
    size_t i = 0;
    f[i++] = 0xFF, f[i++] = 0xD8;
    if (variant < 2) { /* DHT with bits[0] = 3 or 255 (at most 2 codes of length 1) */
      const int n1 = variant == 0 ? 3 : 255;
      f[i++] = 0xFF, f[i++] = 0xC4;
      i = put16(f, i, 2 + 17 + n1);
      f[i++] = 0x00;
      f[i++] = (uint8_t)n1;
      for (int k = 1; k < 16; k++) f[i++] = 0;
      for (int k = 0; k < n1; k++) f[i++] = (uint8_t)k;
    } else { /* 65535 x 65535 x 3 components with a few bytes of data */
      f[i++] = 0xFF, f[i++] = 0xDB;
      i = put16(f, i, 2 + 65);
      f[i++] = 0x00;
      for (int k = 0; k < 64; k++) f[i++] = 1;
      f[i++] = 0xFF, f[i++] = 0xC0;
      i = put16(f, i, 2 + 6 + 9);
      f[i++] = 8;
      i = put16(f, i, 65535);
      i = put16(f, i, 65535);
      f[i++] = 3;
      for (int c = 0; c < 3; c++) f[i++] = (uint8_t)(c + 1), f[i++] = 0x11, f[i++] = 0;
      for (int ac = 0; ac < 2; ac++) { /* one 1-bit code each: DC cat 0, AC EOB */
        f[i++] = 0xFF, f[i++] = 0xC4;
        i = put16(f, i, 2 + 17 + 1);
        f[i++] = (uint8_t)(ac << 4);
        f[i++] = 1;
        for (int k = 1; k < 16; k++) f[i++] = 0;
        f[i++] = 0;
      }
      f[i++] = 0xFF, f[i++] = 0xDA;
      i = put16(f, i, 2 + 1 + 6 + 3);
      f[i++] = 3;
      for (int c = 0; c < 3; c++) f[i++] = (uint8_t)(c + 1), f[i++] = 0x00;
      f[i++] = 0, f[i++] = 63, f[i++] = 0;
      for (int k = 0; k < 32; k++) f[i++] = 0x00;
    }
    f[i++] = 0xFF, f[i++] = 0xD9;
    if (uphip_jpeg_entropy_decode(f, i, NULL, 0) >= 0) {
      fprintf(stderr, "crafted jpeg %d accepted\n", variant);
      g_fail++;
    }
    uphip_clear_error();
  }
}

int main(int argc, char **argv) {
  const char *dir = argc > 1 ? argv[1] : "/tmp";
  UphipOptions o;
  o_options_init(&o);
  for (int fmt = UPHIP_FMT_GRAY8; fmt <= UPHIP_FMT_MONOBLACK; fmt++)
    sheet("default", &o, fmt, 310, 440, 3);
  o.layout = UPHIP_LAYOUT_DOUBLE;
  o.interpolate_type = UPHIP_INTERP_LINEAR;
  sheet("double", &o, UPHIP_FMT_RGB24, 420, 300, 7);
  o.input_count = 2;
  o.output_count = 2;
  sheet("two pages", &o, UPHIP_FMT_GRAY8, 240, 330, 11);
  o_options_init(&o);
  o.interpolate_type = UPHIP_INTERP_NN;
  o.pre_rotate = 90;
  o.post_mirror = (UphipDirection){true, false};
  o.noisefilter_intensity = 9;
  sheet("geometry", &o, UPHIP_FMT_GRAY8, 300, 420, 15);
  codec(dir);
  png(dir, argc > 2 ? argv[2] : "tests/golden/reference");
  jpeg(argc > 2 ? argv[2] : "tests/golden/reference");
  jpeg_crafted();
  j2k(argc > 2 ? argv[2] : "tests/golden/reference");
  pdf(dir, argc > 2 ? argv[2] : "tests/golden/reference");
  printf("sanitize: %d failures\n", g_fail);
  return g_fail ? 1 : 0;
}
