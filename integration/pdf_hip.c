/* pdf_hip.c — pdf/pdf_reader.c and pdf/pdf_writer.c for unpaper-gpu without
 * MuPDF: the reference's PDF reader / writer API (pdf/pdf_reader.h,
 * pdf/pdf_writer.h, as they are) on libunpaper_hip.so's uphip_pdf_*.  A
 * maintainer links this file instead of the two MuPDF-backed sources; the
 * PDF pipelines above them (pdf_pipeline_*.c) are unchanged.
 *
 * pdf_render_page* (pdf_reader.c:443-775, MuPDF's rasteriser) is provided
 * for image pages only: the page's largest image, decoded by
 * uphip_pdf_read_page (JPEG / JPEG 2000 on the device, the rest on the
 * host), scaled to the page's size at `dpi` (or to the target size) by box
 * averaging.  That is what MuPDF draws for a scanned page up to its own
 * resampling filter, so the pixels are not MuPDF's; pages without an image
 * return NULL with the error set.
 *
 * Compiles against the reference headers where they lie
 * (`cc -I<reference> -I<repo>/include -c integration/pdf_hip.c`).
 */
#include <stdarg.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <math.h>

#include "pdf/pdf_reader.h"
#include "pdf/pdf_writer.h"
#include "unpaper_hip.h"

/* the reference's enum values are the C ABI's (pdf_reader.h:19-28) */
#define SAME_VALUE(a, b) _Static_assert((int)(a) == (int)(b), #a)
SAME_VALUE(PDF_IMAGE_UNKNOWN, UPHIP_PDF_IMAGE_UNKNOWN);
SAME_VALUE(PDF_IMAGE_JPEG, UPHIP_PDF_IMAGE_JPEG);
SAME_VALUE(PDF_IMAGE_JP2, UPHIP_PDF_IMAGE_JP2);
SAME_VALUE(PDF_IMAGE_JBIG2, UPHIP_PDF_IMAGE_JBIG2);
SAME_VALUE(PDF_IMAGE_CCITT, UPHIP_PDF_IMAGE_CCITT);
SAME_VALUE(PDF_IMAGE_PNG, UPHIP_PDF_IMAGE_PNG);
SAME_VALUE(PDF_IMAGE_RAW, UPHIP_PDF_IMAGE_RAW);
SAME_VALUE(PDF_IMAGE_FLATE, UPHIP_PDF_IMAGE_FLATE);
_Static_assert(sizeof(PdfMetadata) == sizeof(UphipPdfMetadata), "PdfMetadata");

struct PdfDocument {
  UphipPdfDocument *doc;
};
struct PdfWriter {
  UphipPdfWriter *w;
  int dpi;
};

static __thread char last_error[512];

static void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(last_error, sizeof(last_error), fmt, ap);
  va_end(ap);
}

/* the library's error, moved into this file's (pdf_get_last_error) */
static void take_error(const char *what) {
  const char *e = uphip_last_error();
  set_error("%s%s%s", what, e ? ": " : "", e ? e : "");
  uphip_clear_error();
}

const char *pdf_get_last_error(void) { return last_error; }
const char *pdf_writer_get_last_error(void) { return last_error; }

const char *pdf_image_format_name(PdfImageFormat format) { return uphip_pdf_image_format_name((int32_t)format); }

bool pdf_is_pdf_file(const char *filename) { return uphip_pdf_is_pdf_file(filename) != 0; }

static PdfDocument *wrap(UphipPdfDocument *d, const char *what) {
  if (!d) {
    take_error(what);
    return NULL;
  }
  PdfDocument *p = calloc(1, sizeof(*p));
  if (!p) {
    uphip_pdf_close(d);
    set_error("Out of memory");
    return NULL;
  }
  p->doc = d;
  return p;
}

PdfDocument *pdf_open(const char *path) {
  if (!path) {
    set_error("NULL path");
    return NULL;
  }
  return wrap(uphip_pdf_open(path), "Failed to open document");
}

PdfDocument *pdf_open_memory(const uint8_t *data, size_t size) {
  if (!data || !size) {
    set_error("Invalid data");
    return NULL;
  }
  return wrap(uphip_pdf_open_memory(data, size), "Failed to open document from memory");
}

void pdf_close(PdfDocument *doc) {
  if (!doc) return;
  uphip_pdf_close(doc->doc);
  free(doc);
}

int pdf_page_count(PdfDocument *doc) { return doc ? uphip_pdf_page_count(doc->doc) : -1; }

bool pdf_doc_needs_password(PdfDocument *doc) { return doc && uphip_pdf_needs_password(doc->doc); }

bool pdf_doc_authenticate(PdfDocument *doc, const char *password) {
  (void)password;
  if (!doc) return false;
  if (!uphip_pdf_needs_password(doc->doc)) return true;  /* nothing to unlock */
  set_error("Encrypted PDFs are not supported (no decryption)");
  return false;
}

bool pdf_get_page_info(PdfDocument *doc, int page, PdfPageInfo *info) {
  if (!doc || !info) {
    set_error("Invalid arguments");
    return false;
  }
  UphipPdfPageInfo u;
  if (uphip_pdf_get_page_info(doc->doc, page, &u) != 0) {
    take_error("Failed to get page info");
    return false;
  }
  info->width = u.width;
  info->height = u.height;
  info->rotation = u.rotation;
  return true;
}

bool pdf_extract_page_image(PdfDocument *doc, int page, PdfImage *image) {
  if (!doc || !image) {
    set_error("Invalid arguments");
    return false;
  }
  memset(image, 0, sizeof(*image));
  UphipPdfImage u;
  if (uphip_pdf_extract_page_image(doc->doc, page, &u) != 0) {
    take_error("Failed to extract image");
    return false;
  }
  /* the bytes are malloc'd by the library: ownership passes to the caller
   * (pdf_free_image frees them) */
  image->data = u.data;
  image->size = u.size;
  image->width = u.width;
  image->height = u.height;
  image->components = u.components;
  image->bits_per_component = u.bits_per_component;
  image->format = (PdfImageFormat)u.format;
  image->is_mask = u.is_mask != 0;
  image->jbig2_globals = u.jbig2_globals;
  image->jbig2_globals_size = u.jbig2_globals_size;
  return true;
}

void pdf_free_image(PdfImage *image) {
  if (!image) return;
  free(image->data);
  free(image->jbig2_globals);
  memset(image, 0, sizeof(*image));
}

/* ---- rendering of image pages ---------------------------------------- */

/* the page image as RGB24 or GRAY8 host pixels (channels 3 or 1) */
static uint8_t *page_pixels(PdfDocument *doc, int page, int *w, int *h, int *channels) {
  UphipPnmInfo g;
  if (uphip_pdf_page_probe(doc->doc, page, 0, &g) != 0) {
    take_error("Failed to render page (pages without an image need a rasteriser)");
    return NULL;
  }
  const int64_t ls = g.format == UPHIP_FMT_RGB24 ? 3 * (int64_t)g.width
                     : g.format == UPHIP_FMT_GRAY8 ? g.width : ((int64_t)g.width + 7) / 8;
  uint8_t *raw = malloc((size_t)(ls * g.height));
  if (!raw) {
    set_error("Out of memory");
    return NULL;
  }
  if (uphip_pdf_read_page(doc->doc, page, 0, raw, ls, &g) != 0) {
    take_error("Failed to render page");
    free(raw);
    return NULL;
  }
  if (g.format == UPHIP_FMT_MONOWHITE || g.format == UPHIP_FMT_MONOBLACK) {
    uint8_t *gray = malloc((size_t)g.width * g.height);
    if (!gray) {
      free(raw);
      set_error("Out of memory");
      return NULL;
    }
    for (int y = 0; y < g.height; y++)
      for (int x = 0; x < g.width; x++) {
        const int bit = raw[(int64_t)y * ls + (x >> 3)] >> (7 - (x & 7)) & 1;
        /* monowhite: 1 is black; monoblack: 1 is white */
        gray[(int64_t)y * g.width + x] = (uint8_t)((g.format == UPHIP_FMT_MONOWHITE) ^ bit ? 255 : 0);
      }
    free(raw);
    raw = gray;
    *channels = 1;
  } else {
    *channels = g.format == UPHIP_FMT_RGB24 ? 3 : 1;
  }
  *w = g.width;
  *h = g.height;
  return raw;
}

/* box-average resampling of a (w, h, sc channels) image to (tw, th) with dc
 * output channels (gray -> rgb replicates, rgb -> gray as (r+g+b)/3) */
static uint8_t *resample(const uint8_t *src, int w, int h, int sc, int tw, int th, int dc) {
  uint8_t *dst = malloc((size_t)tw * th * dc);
  if (!dst) return NULL;
  for (int ty = 0; ty < th; ty++) {
    const int y0 = (int)((int64_t)ty * h / th), y1 = (int)(((int64_t)ty + 1) * h / th);
    const int ye = y1 > y0 ? y1 : y0 + 1;
    for (int tx = 0; tx < tw; tx++) {
      const int x0 = (int)((int64_t)tx * w / tw), x1 = (int)(((int64_t)tx + 1) * w / tw);
      const int xe = x1 > x0 ? x1 : x0 + 1;
      uint64_t acc[3] = {0, 0, 0};
      for (int y = y0; y < ye && y < h; y++)
        for (int x = x0; x < xe && x < w; x++)
          for (int c = 0; c < sc; c++) acc[c] += src[((int64_t)y * w + x) * sc + c];
      const uint64_t n = (uint64_t)((ye < h ? ye : h) - y0) * (uint64_t)((xe < w ? xe : w) - x0);
      uint8_t *o = dst + ((int64_t)ty * tw + tx) * dc;
      if (sc == dc) {
        for (int c = 0; c < dc; c++) o[c] = (uint8_t)((acc[c] + n / 2) / n);
      } else if (dc == 3) {
        o[0] = o[1] = o[2] = (uint8_t)((acc[0] + n / 2) / n);
      } else {
        o[0] = (uint8_t)((acc[0] + acc[1] + acc[2] + 3 * n / 2) / (3 * n));
      }
    }
  }
  return dst;
}

static uint8_t *render(PdfDocument *doc, int page, int dpi, int tw, int th, int dc, int *width, int *height,
                       int *stride) {
  if (!doc || !width || !height || !stride) {
    set_error("Invalid arguments");
    return NULL;
  }
  if (tw <= 0 || th <= 0) {
    PdfPageInfo info;
    if (dpi <= 0 || !pdf_get_page_info(doc, page, &info)) {
      if (dpi <= 0) set_error("Invalid DPI: %d", dpi);
      return NULL;
    }
    tw = (int)lroundf(info.width * (float)dpi / 72.0f);
    th = (int)lroundf(info.height * (float)dpi / 72.0f);
    if (tw <= 0 || th <= 0) {
      set_error("Invalid page size");
      return NULL;
    }
  }
  int w, h, sc;
  uint8_t *px = page_pixels(doc, page, &w, &h, &sc);
  if (!px) return NULL;
  uint8_t *out = resample(px, w, h, sc, tw, th, dc);
  free(px);
  if (!out) {
    set_error("Out of memory");
    return NULL;
  }
  *width = tw;
  *height = th;
  *stride = tw * dc;
  return out;
}

uint8_t *pdf_render_page(PdfDocument *doc, int page, int dpi, int *width, int *height, int *stride) {
  return render(doc, page, dpi, 0, 0, 3, width, height, stride);
}

uint8_t *pdf_render_page_gray(PdfDocument *doc, int page, int dpi, int *width, int *height, int *stride) {
  return render(doc, page, dpi, 0, 0, 1, width, height, stride);
}

uint8_t *pdf_render_page_to_size(PdfDocument *doc, int page, int target_width, int target_height, int *width,
                                 int *height, int *stride) {
  if (target_width <= 0 || target_height <= 0) {
    set_error("Invalid target size");
    return NULL;
  }
  return render(doc, page, 0, target_width, target_height, 3, width, height, stride);
}

uint8_t *pdf_render_page_gray_to_size(PdfDocument *doc, int page, int target_width, int target_height,
                                      int *width, int *height, int *stride) {
  if (target_width <= 0 || target_height <= 0) {
    set_error("Invalid target size");
    return NULL;
  }
  return render(doc, page, 0, target_width, target_height, 1, width, height, stride);
}

/* ---- metadata --------------------------------------------------------- */

PdfMetadata pdf_get_metadata(PdfDocument *doc) {
  PdfMetadata m;
  memset(&m, 0, sizeof(m));
  UphipPdfMetadata u;
  if (!doc || uphip_pdf_get_metadata(doc->doc, &u) != 0) {
    uphip_clear_error();
    return m;
  }
  /* the same eight malloc'd strings, same order (pdf_reader.h:47-56) */
  memcpy(&m, &u, sizeof(m));
  return m;
}

void pdf_free_metadata(PdfMetadata *meta) { uphip_pdf_free_metadata((UphipPdfMetadata *)meta); }

/* ---- writer ----------------------------------------------------------- */

PdfWriter *pdf_writer_create(const char *path, const PdfMetadata *meta, int dpi) {
  if (!path) {
    set_error("NULL path");
    return NULL;
  }
  UphipPdfWriter *w = uphip_pdf_writer_create(path, (const UphipPdfMetadata *)meta, dpi);
  if (!w) {
    take_error("Failed to create PDF document");
    return NULL;
  }
  PdfWriter *p = calloc(1, sizeof(*p));
  if (!p) {
    uphip_pdf_writer_abort(w);
    set_error("Out of memory");
    return NULL;
  }
  p->w = w;
  p->dpi = dpi > 0 ? dpi : 72;
  return p;
}

bool pdf_writer_close(PdfWriter *writer) {
  if (!writer) return true;
  const int rc = uphip_pdf_writer_close(writer->w);
  if (rc != 0) take_error("Failed to save PDF");
  free(writer);
  return rc == 0;
}

void pdf_writer_abort(PdfWriter *writer) {
  if (!writer) return;
  uphip_pdf_writer_abort(writer->w);
  free(writer);
}

bool pdf_writer_add_page_jpeg(PdfWriter *writer, const uint8_t *data, size_t len, int width, int height, int dpi) {
  if (!writer || !data || !len) {
    set_error("Invalid arguments");
    return false;
  }
  if (uphip_pdf_writer_add_page_jpeg(writer->w, data, len, width, height, dpi) != 0) {
    take_error("Failed to add JPEG page");
    return false;
  }
  return true;
}

bool pdf_writer_add_page_jp2(PdfWriter *writer, const uint8_t *data, size_t len, int width, int height, int dpi) {
  if (!writer || !data || !len) {
    set_error("Invalid arguments");
    return false;
  }
  if (uphip_pdf_writer_add_page_jp2(writer->w, data, len, width, height, dpi) != 0) {
    take_error("Failed to add JP2 page");
    return false;
  }
  return true;
}

bool pdf_writer_add_page_pixels(PdfWriter *writer, const uint8_t *pixels, int width, int height, int stride,
                                PdfPixelFormat format, int dpi) {
  if (!writer || !pixels) {
    set_error("Invalid arguments");
    return false;
  }
  if (uphip_pdf_writer_add_page_pixels(writer->w, pixels, width, height, stride,
                                       format == PDF_PIXEL_GRAY8 ? 0 : 1, dpi) != 0) {
    take_error("Failed to add pixel page");
    return false;
  }
  return true;
}

int pdf_writer_page_count(const PdfWriter *writer) { return writer ? uphip_pdf_writer_page_count(writer->w) : 0; }
