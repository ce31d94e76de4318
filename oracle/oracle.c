/*
 * oracle.c — CPU restatement of the reference CPU path. TEST INFRASTRUCTURE:
 * the product never links this file; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it (see oracle.h).
 *
 * Every function names the reference function and file:line it restates
 * (paths relative to ErrorTzy/unpaper-gpu @ 2026-01-30).  Arithmetic types,
 * evaluation order and float expressions are kept as in the reference so the
 * results are bit-identical; build with FP contraction off (Makefile).
 *
 * One deliberate structural difference: flood_fill (fill.c:81-107) recurses
 * without bound in the reference; here the recursion is run on an explicit
 * heap stack that visits calls in exactly the same order (same result, no
 * stack overflow on large dark regions).
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define OMAX(a, b) ((a) > (b) ? (a) : (b))
#define OMIN(a, b) ((a) < (b) ? (a) : (b))

static const UphipPixel PX_WHITE = {255, 255, 255};
static const UphipPixel PX_BLACK = {0, 0, 0};

static OStats g_stats;
void o_stats_get(OStats *out) { *out = g_stats; }
void o_stats_reset(void) { memset(&g_stats, 0, sizeof(g_stats)); }

/* ------------------------------------------------------------------------
 * primitives.c
 * ---------------------------------------------------------------------- */
static inline UphipRectangle rect_from_size(UphipPoint o, UphipRectangleSize s) {
  /* rectangle_from_size, primitives.c:26-37 */
  UphipRectangle r = {{o, {o.x + s.width - 1, o.y + s.height - 1}}};
  return r;
}

static inline UphipRectangleSize rect_size(UphipRectangle r) {
  /* size_of_rectangle, primitives.c:39-44 */
  UphipRectangleSize s = {abs(r.vertex[0].x - r.vertex[1].x) + 1,
                          abs(r.vertex[0].y - r.vertex[1].y) + 1};
  return s;
}

static inline UphipRectangle rect_normalize(UphipRectangle in) {
  /* normalize_rectangle, primitives.c:46-61 */
  UphipRectangle r = {{{OMIN(in.vertex[0].x, in.vertex[1].x),
                        OMIN(in.vertex[0].y, in.vertex[1].y)},
                       {OMAX(in.vertex[0].x, in.vertex[1].x),
                        OMAX(in.vertex[0].y, in.vertex[1].y)}}};
  return r;
}

static inline UphipRectangle rect_shift(UphipRectangle r, UphipDelta d) {
  /* shift_rectangle, primitives.c:63-68 */
  r.vertex[0].x += d.horizontal;
  r.vertex[0].y += d.vertical;
  r.vertex[1].x += d.horizontal;
  r.vertex[1].y += d.vertical;
  return r;
}

static inline uint64_t rect_count(UphipRectangle r) {
  /* count_pixels, primitives.c:88-92: int32 product widened */
  UphipRectangleSize s = rect_size(r);
  return (uint64_t)(s.width * s.height);
}

static inline bool point_in(UphipPoint p, UphipRectangle in) {
  /* point_in_rectangle, primitives.c:94-99 */
  UphipRectangle a = rect_normalize(in);
  return p.x >= a.vertex[0].x && p.x <= a.vertex[1].x && p.y >= a.vertex[0].y &&
         p.y <= a.vertex[1].y;
}

static bool rects_overlap(UphipRectangle first_in, UphipRectangle second_in) {
  /* rectangles_overlap, primitives.c:117-123: only first's two corners */
  UphipRectangle a = rect_normalize(first_in);
  UphipRectangle b = rect_normalize(second_in);
  return point_in(a.vertex[0], b) || point_in(a.vertex[1], b);
}

static int compare_sizes(UphipRectangleSize a, UphipRectangleSize b) {
  /* compare_sizes, primitives.c:70-80 */
  if (a.height == b.height && a.width == b.width) return 0;
  return OMIN(a.height, a.width) < OMIN(b.height, b.width) ? -1 : 1;
}

static UphipRectangleSize coerce_size(UphipRectangleSize s, UphipRectangleSize d) {
  /* coerce_size, primitives.c:82-86 */
  UphipRectangleSize r = {s.width == -1 ? d.width : s.width,
                          s.height == -1 ? d.height : s.height};
  return r;
}

/* ------------------------------------------------------------------------
 * image.c
 * ---------------------------------------------------------------------- */
static inline UphipRectangleSize image_size(OImage im) {
  UphipRectangleSize s = {im.width, im.height};
  return s;
}
static inline UphipRectangle full_image(OImage im) {
  UphipPoint o = {0, 0};
  return rect_from_size(o, image_size(im));
}

static UphipRectangle clip_rect(OImage im, UphipRectangle area) {
  /* clip_rectangle, image.c:72-88 */
  UphipRectangle n = rect_normalize(area);
  UphipRectangle r = {{{OMAX(n.vertex[0].x, 0), OMAX(n.vertex[0].y, 0)},
                       {OMIN(n.vertex[1].x, im.width - 1),
                        OMIN(n.vertex[1].y, im.height - 1)}}};
  return r;
}

int64_t o_min_linesize(int32_t width, int32_t format) {
  switch (format) {
  case UPHIP_FMT_GRAY8: return width;
  case UPHIP_FMT_Y400A: return 2 * (int64_t)width;
  case UPHIP_FMT_RGB24: return 3 * (int64_t)width;
  default: return ((int64_t)width + 7) / 8;
  }
}

OImage o_create_image(UphipRectangleSize size, int32_t format, bool fill,
                      UphipPixel background, uint8_t abs_black_threshold) {
  /* create_image, image.c:19-44 (8-byte aligned rows) */
  OImage im;
  im.width = size.width;
  im.height = size.height;
  im.format = format;
  im.linesize = (o_min_linesize(size.width, format) + 7) & ~(int64_t)7;
  im.background = background;
  im.abs_black_threshold = abs_black_threshold;
  size_t bytes = (size_t)im.linesize * (size_t)(size.height > 0 ? size.height : 0);
  im.data = (uint8_t *)calloc(bytes ? bytes : 1, 1);
  if (fill) o_wipe_rectangle(im, full_image(im), background);
  return im;
}

void o_free_image(OImage *im) {
  free(im->data);
  im->data = NULL;
}

static void replace_image(OImage *im, OImage *n) {
  /* replace_image, image.c:46-50 */
  o_free_image(im);
  *im = *n;
  n->data = NULL;
}

static OImage create_compatible(OImage src, UphipRectangleSize size, bool fill) {
  /* create_compatible_image, image.c:56-59 */
  return o_create_image(size, src.format, fill, src.background,
                        src.abs_black_threshold);
}

/* ------------------------------------------------------------------------
 * pixel.c
 * ---------------------------------------------------------------------- */
static inline uint8_t px_gray(UphipPixel p) {
  /* pixel_grayscale, pixel.c:16-18 */
  return (uint8_t)((p.r + p.g + p.b) / 3);
}

UphipPixel o_get_pixel(OImage im, UphipPoint c) {
  /* get_pixel_components, pixel.c:20-63: outside the image reads WHITE */
  if (c.x < 0 || c.y < 0 || c.x >= im.width || c.y >= im.height) return PX_WHITE;
  const uint8_t *row = im.data + (int64_t)c.y * im.linesize;
  UphipPixel r;
  switch (im.format) {
  case UPHIP_FMT_GRAY8:
    r.r = r.g = r.b = row[c.x];
    return r;
  case UPHIP_FMT_Y400A:
    r.r = r.g = r.b = row[2 * c.x];
    return r;
  case UPHIP_FMT_RGB24:
    r.r = row[3 * c.x];
    r.g = row[3 * c.x + 1];
    r.b = row[3 * c.x + 2];
    return r;
  case UPHIP_FMT_MONOWHITE:
    return (row[c.x / 8] & (128 >> (c.x % 8))) ? PX_BLACK : PX_WHITE;
  case UPHIP_FMT_MONOBLACK:
    return (row[c.x / 8] & (128 >> (c.x % 8))) ? PX_WHITE : PX_BLACK;
  default:
    return PX_WHITE;
  }
}

static inline uint8_t get_gray(OImage im, UphipPoint c) {
  return px_gray(o_get_pixel(im, c)); /* get_pixel_grayscale, pixel.c:85-87 */
}
static inline uint8_t get_lightness(OImage im, UphipPoint c) {
  UphipPixel p = o_get_pixel(im, c); /* get_pixel_lightness, pixel.c:101-104 */
  uint8_t m = p.r < p.g ? p.r : p.g;
  return m < p.b ? m : p.b;
}
static inline uint8_t get_darkness_inverse(OImage im, UphipPoint c) {
  UphipPixel p = o_get_pixel(im, c); /* pixel.c:118-121 */
  uint8_t m = p.r > p.g ? p.r : p.g;
  return m > p.b ? m : p.b;
}

void o_set_pixel(OImage im, UphipPoint c, UphipPixel px) {
  /* set_pixel, pixel.c:126-173: writes outside the image are dropped */
  if (c.x < 0 || c.y < 0 || c.x >= im.width || c.y >= im.height) return;
  bool black = px_gray(px) < im.abs_black_threshold;
  uint8_t *row = im.data + (int64_t)c.y * im.linesize;
  switch (im.format) {
  case UPHIP_FMT_GRAY8:
    row[c.x] = px_gray(px);
    break;
  case UPHIP_FMT_Y400A:
    row[2 * c.x] = px_gray(px);
    row[2 * c.x + 1] = 0xFF;
    break;
  case UPHIP_FMT_RGB24:
    row[3 * c.x] = px.r;
    row[3 * c.x + 1] = px.g;
    row[3 * c.x + 2] = px.b;
    break;
  case UPHIP_FMT_MONOWHITE:
    black = !black; /* fallthrough: inverted sense */
  case UPHIP_FMT_MONOBLACK:
    if (!black)
      row[c.x / 8] |= (uint8_t)(128 >> (c.x % 8));
    else
      row[c.x / 8] &= (uint8_t)~(128 >> (c.x % 8));
    break;
  default:
    break;
  }
}

/* ------------------------------------------------------------------------
 * blit.c
 * ---------------------------------------------------------------------- */
void o_wipe_rectangle(OImage im, UphipRectangle input_area, UphipPixel color) {
  /* wipe_rectangle_cpu, blit.c:20-24 */
  UphipRectangle a = clip_rect(im, input_area);
  for (int32_t y = a.vertex[0].y; y <= a.vertex[1].y; y++)
    for (int32_t x = a.vertex[0].x; x <= a.vertex[1].x; x++)
      o_set_pixel(im, (UphipPoint){x, y}, color);
}

void o_copy_rectangle(OImage src, OImage dst, UphipRectangle source_area,
                      UphipPoint tc) {
  /* copy_rectangle_cpu, blit.c:30-80.  The memcpy fast path (same byte
   * format, whole target rectangle inside the target) copies raw bytes, which
   * differs from the per-pixel path only for Y400A: set_pixel writes alpha
   * 0xFF, memcpy keeps the source alpha. */
  UphipRectangle a = clip_rect(src, source_area);
  const int32_t w = a.vertex[1].x - a.vertex[0].x + 1;
  const int32_t h = a.vertex[1].y - a.vertex[0].y + 1;
  const int bpp = src.format == UPHIP_FMT_GRAY8 ? 1 : src.format == UPHIP_FMT_Y400A ? 2
                  : src.format == UPHIP_FMT_RGB24 ? 3 : 0;
  if (src.format == dst.format && w > 0 && h > 0 && tc.x >= 0 && tc.y >= 0 &&
      tc.x + w <= dst.width && tc.y + h <= dst.height && bpp > 0) {
    for (int32_t sy = a.vertex[0].y, ty = tc.y; sy <= a.vertex[1].y; sy++, ty++)
      memcpy(dst.data + (int64_t)ty * dst.linesize + (int64_t)tc.x * bpp,
             src.data + (int64_t)sy * src.linesize + (int64_t)a.vertex[0].x * bpp,
             (size_t)w * bpp);
    return;
  }
  for (int32_t sy = a.vertex[0].y, ty = tc.y; sy <= a.vertex[1].y; sy++, ty++)
    for (int32_t sx = a.vertex[0].x, tx = tc.x; sx <= a.vertex[1].x; sx++, tx++)
      o_set_pixel(dst, (UphipPoint){tx, ty}, o_get_pixel(src, (UphipPoint){sx, sy}));
}

static uint8_t inverse_brightness_rect(OImage im, UphipRectangle input_area) {
  /* blit.c:91-109 */
  uint64_t sum = 0;
  UphipRectangle a = clip_rect(im, input_area);
  uint64_t count = rect_count(a);
  if (count == 0) return 0;
  for (int32_t y = a.vertex[0].y; y <= a.vertex[1].y; y++)
    for (int32_t x = a.vertex[0].x; x <= a.vertex[1].x; x++)
      sum += get_gray(im, (UphipPoint){x, y});
  return (uint8_t)(0xFF - (sum / count));
}

static uint8_t inverse_lightness_rect(OImage im, UphipRectangle input_area) {
  /* blit.c:111-129 */
  uint64_t sum = 0;
  UphipRectangle a = clip_rect(im, input_area);
  uint64_t count = rect_count(a);
  if (count == 0) return 0;
  for (int32_t y = a.vertex[0].y; y <= a.vertex[1].y; y++)
    for (int32_t x = a.vertex[0].x; x <= a.vertex[1].x; x++)
      sum += get_lightness(im, (UphipPoint){x, y});
  return (uint8_t)(0xFF - (sum / count));
}

static uint8_t darkness_rect(OImage im, UphipRectangle input_area) {
  /* blit.c:131-146 */
  uint64_t sum = 0;
  UphipRectangle a = clip_rect(im, input_area);
  uint64_t count = rect_count(a);
  if (count == 0) return 0;
  for (int32_t y = a.vertex[0].y; y <= a.vertex[1].y; y++)
    for (int32_t x = a.vertex[0].x; x <= a.vertex[1].x; x++)
      sum += get_darkness_inverse(im, (UphipPoint){x, y});
  return (uint8_t)(0xFF - (sum / count));
}

static uint64_t count_within_brightness(OImage im, UphipRectangle area,
                                        uint8_t lo, uint8_t hi, bool clear) {
  /* count_pixels_within_brightness, blit.c:148-173 (area NOT clipped) */
  uint64_t count = 0;
  for (int32_t y = area.vertex[0].y; y <= area.vertex[1].y; y++)
    for (int32_t x = area.vertex[0].x; x <= area.vertex[1].x; x++) {
      UphipPoint p = {x, y};
      uint8_t b = get_gray(im, p);
      if (b < lo || b > hi) continue;
      if (clear) o_set_pixel(im, p, PX_WHITE);
      count++;
    }
  return count;
}

void o_center_image(OImage src, OImage dst, UphipPoint to,
                    UphipRectangleSize ts) {
  /* center_image_cpu, blit.c:175-202 */
  UphipPoint so = {0, 0};
  UphipRectangleSize ss = image_size(src);
  if (ss.width < ts.width || ss.height < ts.height)
    o_wipe_rectangle(dst, rect_from_size(to, ts), dst.background);
  if (ss.width <= ts.width) {
    to.x += (ts.width - ss.width) / 2;
  } else {
    so.x += (ss.width - ts.width) / 2;
    ss.width = ts.width;
  }
  if (ss.height <= ts.height) {
    to.y += (ts.height - ss.height) / 2;
  } else {
    so.y += (ss.height - ts.height) / 2;
    ss.height = ts.height;
  }
  o_copy_rectangle(src, dst, rect_from_size(so, ss), to);
}

/* interpolate.c */
static UphipPixel interp_nn(OImage im, float cx, float cy) {
  /* interp_nearest_neighbour, interpolate.c:13-18 */
  UphipPoint p = {(int)roundf(cx), (int)roundf(cy)};
  return o_get_pixel(im, p);
}

static uint8_t cubic_scale(float factor, uint8_t a, uint8_t b, uint8_t c,
                           uint8_t d) {
  /* interpolate.c:24-31 (same expression, same association) */
  int result = b + 0.5f * factor *
                       (c - a + factor * (2.0f * a - 5.0f * b + 4.0f * c - d +
                                          factor * (3.0f * (b - c) + d - a)));
  return (uint8_t)(result < 0 ? 0 : (result > 255 ? 255 : result)); /* av_clip_uint8 */
}

static UphipPixel cubic_px(float f, const UphipPixel q[4]) {
  UphipPixel r = {cubic_scale(f, q[0].r, q[1].r, q[2].r, q[3].r),
                  cubic_scale(f, q[0].g, q[1].g, q[2].g, q[3].g),
                  cubic_scale(f, q[0].b, q[1].b, q[2].b, q[3].b)};
  return r;
}

static UphipPixel interp_bicubic(OImage im, float cx, float cy) {
  /* interp_bicubic, interpolate.c:43-60 */
  UphipPoint p = {(int)cx, (int)cy};
  UphipPixel col[4];
  for (int i = -1; i < 3; ++i) {
    UphipPixel q[4] = {o_get_pixel(im, (UphipPoint){p.x - 1, p.y + i}),
                       o_get_pixel(im, (UphipPoint){p.x, p.y + i}),
                       o_get_pixel(im, (UphipPoint){p.x + 1, p.y + i}),
                       o_get_pixel(im, (UphipPoint){p.x + 2, p.y + i})};
    col[i + 1] = cubic_px(cx - p.x, q);
  }
  return cubic_px(cy - p.y, col);
}

static uint8_t linear_scale(float x, uint8_t a, uint8_t b) {
  return (uint8_t)((1.0f - x) * a + x * b); /* interpolate.c:62-65 */
}
static UphipPixel linear_px(float f, UphipPixel a, UphipPixel b) {
  UphipPixel r = {linear_scale(f, a.r, b.r), linear_scale(f, a.g, b.g),
                  linear_scale(f, a.b, b.b)};
  return r;
}

static UphipPixel interp_bilinear(OImage im, float cx, float cy) {
  /* interp_bilinear, interpolate.c:77-118 (integral-coordinate quirk kept) */
  UphipRectangle area = full_image(im);
  UphipPoint p1 = {(int)floorf(cx), (int)floorf(cy)};
  UphipPoint p2 = {(int)ceil(cx), (int)ceilf(cy)};
  if (!point_in(p2, area)) return o_get_pixel(im, p1);
  if (p1.x == p2.x && p1.y == p2.y) return o_get_pixel(im, p1);
  if (p1.x == p2.x)
    return linear_px(cx - p1.x, o_get_pixel(im, p1), o_get_pixel(im, p2));
  if (p1.y == p2.y)
    return linear_px(cy - p1.y, o_get_pixel(im, p1), o_get_pixel(im, p2));
  UphipPixel a = o_get_pixel(im, (UphipPoint){p1.x, p1.y});
  UphipPixel b = o_get_pixel(im, (UphipPoint){p2.x, p1.y});
  UphipPixel c = o_get_pixel(im, (UphipPoint){p1.x, p2.y});
  UphipPixel d = o_get_pixel(im, (UphipPoint){p2.x, p2.y});
  UphipPixel h1 = linear_px(cx - p1.x, a, b);
  UphipPixel h2 = linear_px(cx - p1.x, c, d);
  return linear_px(cy - p1.y, h1, h2);
}

static UphipPixel interpolate(OImage im, float cx, float cy, int32_t fn) {
  /* interpolate, interpolate.c:120-129 */
  switch (fn) {
  case UPHIP_INTERP_NN: return interp_nn(im, cx, cy);
  case UPHIP_INTERP_LINEAR: return interp_bilinear(im, cx, cy);
  default: return interp_bicubic(im, cx, cy);
  }
}

static void stretch_frame(OImage src, OImage dst, int32_t interp) {
  /* blit.c:209-229 */
  const float hr = (float)src.width / (float)dst.width;
  const float vr = (float)src.height / (float)dst.height;
  for (int32_t y = 0; y < dst.height; y++)
    for (int32_t x = 0; x < dst.width; x++)
      o_set_pixel(dst, (UphipPoint){x, y}, interpolate(src, x * hr, y * vr, interp));
}

void o_stretch_and_replace(OImage *im, UphipRectangleSize size, int32_t interp) {
  /* blit.c:231-239 */
  if (compare_sizes(image_size(*im), size) == 0) return;
  OImage t = create_compatible(*im, size, false);
  stretch_frame(*im, t, interp);
  replace_image(im, &t);
}

void o_resize_and_replace(OImage *im, UphipRectangleSize size, int32_t interp) {
  /* blit.c:246-282 */
  UphipRectangleSize is = image_size(*im);
  if (compare_sizes(is, size) == 0) return;
  const float hr = (float)size.width / (float)is.width;
  const float vr = (float)size.height / (float)is.height;
  UphipRectangleSize ss;
  if (hr < vr) {
    ss.width = size.width;
    ss.height = (int32_t)(is.height * hr);
  } else if (vr < hr) {
    ss.width = (int32_t)(is.width * vr);
    ss.height = size.height;
  } else {
    ss = size;
  }
  o_stretch_and_replace(im, ss, interp);
  if (size.width == ss.width && size.height == ss.height) return;
  OImage r = create_compatible(*im, size, true);
  o_center_image(*im, r, (UphipPoint){0, 0}, size);
  replace_image(im, &r);
}

void o_flip_rotate_90(OImage *im, int32_t direction) {
  /* flip_rotate_90_cpu, blit.c:289-310 */
  UphipRectangleSize s = image_size(*im);
  UphipRectangleSize ns = {s.height, s.width};
  OImage n = create_compatible(*im, ns, false);
  for (int y = 0; y < s.height; y++) {
    const int xx = ((direction > 0) ? s.height - 1 : 0) - y * direction;
    for (int x = 0; x < s.width; x++) {
      const int yy = ((direction < 0) ? s.width - 1 : 0) + x * direction;
      o_set_pixel(n, (UphipPoint){xx, yy}, o_get_pixel(*im, (UphipPoint){x, y}));
    }
  }
  replace_image(im, &n);
}

void o_mirror(OImage im, UphipDirection d) {
  /* mirror_cpu, blit.c:316-349 */
  UphipRectangle src = {{{0, 0}, {INT32_MAX, INT32_MAX}}};
  UphipRectangleSize s = image_size(im);
  if (d.horizontal && !d.vertical) src.vertex[1].x = (s.width - 1) / 2;
  if (d.vertical) src.vertex[1].y = (s.height - 1) / 2;
  src = clip_rect(im, src);
  for (int32_t y = src.vertex[0].y; y <= src.vertex[1].y; y++) {
    int32_t yy = d.vertical ? s.height - y - 1 : y;
    if (d.vertical && d.horizontal && y == yy) src.vertex[1].x = (s.width - 1) / 2;
    for (int32_t x = 0; x <= src.vertex[1].x; x++) {
      int32_t xx = d.horizontal ? s.width - x - 1 : x;
      UphipPoint p1 = {x, y}, p2 = {xx, yy};
      UphipPixel a = o_get_pixel(im, p1), b = o_get_pixel(im, p2);
      o_set_pixel(im, p1, b);
      o_set_pixel(im, p2, a);
    }
  }
}

void o_shift_image(OImage *im, UphipDelta d) {
  /* shift_image_cpu, blit.c:355-363 */
  OImage n = create_compatible(*im, image_size(*im), true);
  o_copy_rectangle(*im, n, full_image(*im), (UphipPoint){d.horizontal, d.vertical});
  replace_image(im, &n);
}

/* ------------------------------------------------------------------------
 * fill.c — flood fill with the recursion on an explicit stack.
 * ---------------------------------------------------------------------- */
static uint64_t fill_line(OImage im, UphipPoint p, int dx, int dy, UphipPixel color,
                          uint8_t mmin, uint8_t mmax, uint64_t intensity) {
  /* fill_line, fill.c:16-52 */
  uint64_t distance = 0;
  uint64_t icount = 1;
  UphipRectangle area = full_image(im);
  for (;;) {
    p.x += dx;
    p.y += dy;
    uint8_t v = get_gray(im, p);
    if (v >= mmin && v <= mmax)
      icount = intensity;
    else
      icount--;
    if (icount <= 0 || !point_in(p, area)) return distance;
    o_set_pixel(im, p, color);
    distance++;
  }
}

/* direction order of flood_fill (fill.c:92-106): left, up, right, down */
static const int DIR_DX[4] = {-1, 0, 1, 0};
static const int DIR_DY[4] = {0, -1, 0, 1};

typedef struct {
  UphipPoint p;
  uint64_t dist[4];
  int dir;       /* current line being walked around */
  uint64_t d;    /* next position index on that line (0-based) */
  int sub;       /* 0: first neighbour, 1: second neighbour */
} FillFrame;

static bool fill_start(OImage im, UphipPoint p, FillFrame *f, UphipPixel color,
                       uint8_t mmin, uint8_t mmax, uint64_t intensity) {
  /* first half of flood_fill, fill.c:81-96 */
  g_stats.flood_fill_calls++;
  uint8_t v = get_gray(im, p);
  if (!(v >= mmin && v <= mmax)) return false;
  g_stats.flood_fill_matches++;
  o_set_pixel(im, p, color);
  f->p = p;
  for (int k = 0; k < 4; k++)
    f->dist[k] = fill_line(im, p, DIR_DX[k], DIR_DY[k], color, mmin, mmax, intensity);
#ifdef ORACLE_FRAME_LOG
  { /* development aid (tools/dbg/black_frames.sh): one line per frame */
    static FILE *log;
    if (!log && getenv("ORACLE_FRAME_LOG")) log = fopen(getenv("ORACLE_FRAME_LOG"), "w");
    if (log)
      fprintf(log, "%d %d %llu %llu %llu %llu\n", p.x, p.y, (unsigned long long)f->dist[0],
              (unsigned long long)f->dist[1], (unsigned long long)f->dist[2],
              (unsigned long long)f->dist[3]);
  }
#endif
  f->dir = 0;
  f->d = 0;
  f->sub = 0;
  return true;
}

static void flood_fill(OImage im, UphipPoint seed, UphipPixel color, uint8_t mmin,
                       uint8_t mmax, uint64_t intensity) {
  /* flood_fill (fill.c:81-107) + flood_fill_around_line (fill.c:62-79):
   * children of a call are, for each line in order left/up/right/down and
   * each position d = 1..dist along it, the two perpendicular neighbours
   * (horizontal line: below then above; vertical line: right then left). */
  size_t cap = 1024, n = 0;
  FillFrame *st = (FillFrame *)malloc(cap * sizeof(FillFrame));
  if (fill_start(im, seed, &st[0], color, mmin, mmax, intensity)) n = 1;
  while (n > 0) {
    if (n > g_stats.flood_fill_max_depth) g_stats.flood_fill_max_depth = n;
    FillFrame *f = &st[n - 1];
    while (f->dir < 4 && f->d >= f->dist[f->dir]) {
      f->dir++;
      f->d = 0;
      f->sub = 0;
    }
    if (f->dir >= 4) {
      n--;
      continue;
    }
    UphipPoint q = f->p;
    q.x += DIR_DX[f->dir] * (int32_t)(f->d + 1);
    q.y += DIR_DY[f->dir] * (int32_t)(f->d + 1);
    if (DIR_DX[f->dir] != 0) {
      q.y += (f->sub == 0) ? 1 : -1; /* DELTA_DOWNWARD then DELTA_UPWARD */
    } else {
      q.x += (f->sub == 0) ? 1 : -1; /* DELTA_RIGHTWARD then DELTA_LEFTWARD */
    }
    if (f->sub == 0) {
      f->sub = 1;
    } else {
      f->sub = 0;
      f->d++;
    }
    if (n == cap) {
      cap *= 2;
      st = (FillFrame *)realloc(st, cap * sizeof(FillFrame));
    }
    if (fill_start(im, q, &st[n], color, mmin, mmax, intensity)) n++;
  }
  free(st);
}

/* ------------------------------------------------------------------------
 * filters.c
 * ---------------------------------------------------------------------- */
static void blackfilter_scan(OImage im, const UphipBlackfilterParameters *pr,
                             UphipDelta step, UphipRectangleSize stripe,
                             UphipDelta shift) {
  /* blackfilter_scan, filters.c:49-104 (only the first stripe is ever
   * scanned: after the inner loop vertex[0] is past the edge) */
  const UphipRectangle ia = full_image(im);
  UphipRectangle area = rect_from_size((UphipPoint){0, 0}, stripe);
  while (point_in(area.vertex[0], ia)) {
    if (!point_in(area.vertex[1], ia)) {
      UphipDelta d = {ia.vertex[1].x - area.vertex[1].x,
                      ia.vertex[1].y - area.vertex[1].y};
      area = rect_shift(area, d);
    }
    do {
      uint8_t blackness = darkness_rect(im, area);
      if (blackness >= pr->abs_threshold) {
        bool excluded = false;
        for (size_t n = 0; n < pr->exclusions_count; n++)
          if (rects_overlap(area, pr->exclusions[n])) {
            excluded = true;
            break;
          }
        if (!excluded) {
          g_stats.blackfilter_fills++;
          for (int32_t y = area.vertex[0].y; y <= area.vertex[1].y; y++)
            for (int32_t x = area.vertex[0].x; x <= area.vertex[1].x; x++)
              flood_fill(im, (UphipPoint){x, y}, PX_WHITE, 0,
                         im.abs_black_threshold, (uint64_t)pr->intensity);
        }
      }
      area = rect_shift(area, step);
    } while (point_in(area.vertex[0], ia));
    area = rect_shift(area, shift);
  }
}

void o_blackfilter(OImage im, const UphipBlackfilterParameters *pr) {
  /* blackfilter_cpu, filters.c:111-127 */
  if (pr->scan_direction.horizontal)
    blackfilter_scan(im, pr, (UphipDelta){pr->scan_step.horizontal, 0},
                     (UphipRectangleSize){pr->scan_size.width,
                                          (int32_t)pr->scan_depth.vertical},
                     (UphipDelta){0, (int32_t)pr->scan_depth.vertical});
  if (pr->scan_direction.vertical)
    blackfilter_scan(im, pr, (UphipDelta){0, pr->scan_step.vertical},
                     (UphipRectangleSize){(int32_t)pr->scan_depth.horizontal,
                                          pr->scan_size.height},
                     (UphipDelta){(int32_t)pr->scan_depth.horizontal, 0});
}

void o_blurfilter(OImage im, UphipBlurfilterParameters pr, uint8_t white) {
  /* blurfilter_cpu, filters.c:149-232.  The three count rows are pointers
   * into ONE row of the reference's VLA at offsets 0/1/2 and rotate each
   * row; restated literally on a flat array.  Its slot 0 is read before it is
   * written (uninitialised in the reference); zero here. */
  UphipRectangleSize s = image_size(im);
  const uint32_t bpr = (uint32_t)(s.width / pr.scan_size.width);
  const uint64_t total = (uint64_t)(pr.scan_size.width * pr.scan_size.height);
  uint64_t *buf = (uint64_t *)calloc(3 * (size_t)(bpr + 2), sizeof(uint64_t));
  uint64_t *prev = buf + 0, *cur = buf + 1, *next = buf + 2;
  cur[0] = total;
  cur[bpr] = total;
  next[0] = total;
  next[bpr] = total;
  const int32_t max_left = s.width - pr.scan_size.width;
  for (int32_t left = 0, block = 1; left <= max_left; left += pr.scan_size.width)
    cur[block++] = count_within_brightness(
        im, rect_from_size((UphipPoint){left, 0}, pr.scan_size), 0, white, false);
  const int32_t max_top = s.height - pr.scan_size.height;
  for (int32_t top = 0; top <= max_top; top += pr.scan_size.height) {
    next[0] = count_within_brightness(
        im, rect_from_size((UphipPoint){0, top + pr.scan_step.vertical}, pr.scan_size),
        0, white, false);
    for (int32_t left = 0, block = 1; left <= max_left; left += pr.scan_size.width) {
      next[block + 1] = count_within_brightness(
          im,
          rect_from_size((UphipPoint){left + pr.scan_size.width,
                                      top + pr.scan_step.vertical},
                         pr.scan_size),
          0, white, false);
      uint64_t a = prev[block - 1], b = prev[block + 1], c = cur[block];
      uint64_t m1 = a > b ? (a > c ? a : c) : (b > c ? b : c);
      uint64_t d = next[block - 1], e = next[block + 1];
      uint64_t mx = d > e ? (d > m1 ? d : m1) : (e > m1 ? e : m1);
      if ((((float)mx) / total) <= pr.intensity) {
        o_wipe_rectangle(im, rect_from_size((UphipPoint){left, top}, pr.scan_size),
                         PX_WHITE);
        cur[block] = total;
      }
      block++;
    }
    uint64_t *t = prev;
    prev = cur;
    cur = next;
    next = t;
  }
  free(buf);
}

static bool noise_cmp_clear(OImage im, UphipPoint p, bool clear, uint8_t white) {
  /* noisefilter_compare_and_clear, filters.c:238-249 */
  if (get_lightness(im, p) >= white) return false;
  if (clear) o_set_pixel(im, p, PX_WHITE);
  return true;
}

static uint64_t noise_ring(OImage im, UphipPoint p, uint32_t level, bool clear,
                           uint8_t white) {
  /* noisefilter_count_pixel_neighbors_level, filters.c:251-276.
   * `level` is uint32_t there, so `xx <= p.x + level` compares as unsigned:
   * when p.x < level the start value is negative, converts to a huge
   * unsigned and the row loop runs ZERO times (same for the column loop when
   * p.y < level - 1).  Restated with the same conversions. */
  uint64_t count = 0;
  for (int32_t xx = (int32_t)((uint32_t)p.x - level);
       (uint32_t)xx <= (uint32_t)p.x + level; xx++) {
    UphipPoint up = {xx, (int32_t)((uint32_t)p.y - level)};
    UphipPoint lo = {xx, (int32_t)((uint32_t)p.y + level)};
    count += noise_cmp_clear(im, up, clear, white) ? 1 : 0;
    count += noise_cmp_clear(im, lo, clear, white) ? 1 : 0;
  }
  for (int32_t yy = (int32_t)((uint32_t)p.y - (level - 1));
       (uint32_t)yy <= (uint32_t)p.y + (level - 1); yy++) {
    UphipPoint first = {(int32_t)((uint32_t)p.x - level), yy};
    UphipPoint last = {(int32_t)((uint32_t)p.x + level), yy};
    count += noise_cmp_clear(im, first, clear, white) ? 1 : 0;
    count += noise_cmp_clear(im, last, clear, white) ? 1 : 0;
  }
  return count;
}

void o_noisefilter(OImage im, uint64_t intensity, uint8_t white) {
  /* noisefilter_cpu, filters.c:309-338 with the helpers at :278-307 */
  for (int32_t y = 0; y < im.height; y++)
    for (int32_t x = 0; x < im.width; x++) {
      UphipPoint p = {x, y};
      if (get_darkness_inverse(im, p) >= white) continue;
      uint64_t count = 1, lc;
      uint32_t level = 1;
      do {
        lc = noise_ring(im, p, level, false, white);
        count += lc;
        level++;
      } while (lc != 0 && level <= intensity);
      if (count <= intensity) {
        g_stats.noise_clusters++;
        o_set_pixel(im, p, PX_WHITE);
        level = 1;
        do {
          lc = noise_ring(im, p, level, true, white);
          level++;
        } while (lc != 0);
      }
    }
}

void o_grayfilter(OImage im, UphipGrayfilterParameters pr) {
  /* grayfilter_cpu, filters.c:370-402 */
  UphipRectangleSize s = image_size(im);
  UphipPoint o = {0, 0};
  do {
    UphipRectangle area = rect_from_size(o, pr.scan_size);
    uint64_t count = count_within_brightness(im, area, 0, im.abs_black_threshold, false);
    if (count == 0) {
      uint8_t l = inverse_lightness_rect(im, area);
      if (l < pr.abs_threshold) o_wipe_rectangle(im, area, PX_WHITE);
    }
    if (o.x < s.width) {
      o.x += pr.scan_step.horizontal;
    } else {
      o.x = 0;
      o.y += pr.scan_step.vertical;
    }
  } while (o.y <= s.height);
}

/* ------------------------------------------------------------------------
 * masks.c
 * ---------------------------------------------------------------------- */
static uint32_t detect_edge(OImage im, UphipPoint origin, UphipDelta step,
                            int32_t scan_size, int32_t scan_depth, float threshold) {
  /* detect_edge, masks.c:54-100.  The reference loops forever when the bar
   * leaves the image while every bar kept blackness > 0 (a fully outside bar
   * clips to an inverted rectangle and reads 255); here the scan stops once
   * the bar is entirely outside the image (documented divergence). */
  UphipRectangle a;
  UphipRectangleSize s = image_size(im);
  if (step.vertical == 0) {
    if (scan_depth == -1) scan_depth = s.height;
    a = rect_from_size((UphipPoint){origin.x - scan_size / 2, origin.y - scan_depth / 2},
                       (UphipRectangleSize){scan_size, scan_depth});
  } else {
    if (scan_depth == -1) scan_depth = s.width;
    a = rect_from_size((UphipPoint){origin.x - scan_depth / 2, origin.y - scan_size / 2},
                       (UphipRectangleSize){scan_depth, scan_size});
  }
  uint32_t total = 0, count = 0;
  uint8_t blackness;
  do {
    UphipRectangle n = rect_normalize(a);
    bool outside = n.vertex[1].x < 0 || n.vertex[1].y < 0 || n.vertex[0].x >= s.width ||
                   n.vertex[0].y >= s.height;
    blackness = inverse_brightness_rect(im, a); /* 255 for a fully outside bar */
    total += blackness;
    count++;
    a = rect_shift(a, step);
    /* reference would never leave this loop (255 >= threshold*avg forever
     * when threshold <= 1); bounded guard for threshold > 1 */
    if (outside && (threshold <= 1.0f || count >= (1u << 20))) break;
  } while ((blackness >= ((threshold * total) / count)) && blackness != 0);
  return count;
}

static bool detect_mask(OImage im, const UphipMaskDetectionParameters *pr,
                        UphipPoint origin, UphipRectangle *mask) {
  /* detect_mask, masks.c:107-171 */
  UphipRectangleSize s = image_size(im);
  if (pr->scan_direction.horizontal) {
    int32_t le = (int32_t)detect_edge(im, origin, (UphipDelta){-pr->scan_step.horizontal, 0},
                                      pr->scan_size.width, pr->scan_depth.horizontal,
                                      pr->scan_threshold.horizontal);
    int32_t re = (int32_t)detect_edge(im, origin, (UphipDelta){pr->scan_step.horizontal, 0},
                                      pr->scan_size.width, pr->scan_depth.horizontal,
                                      pr->scan_threshold.horizontal);
    mask->vertex[0].x = origin.x - (pr->scan_step.horizontal * le) - pr->scan_size.width / 2;
    mask->vertex[1].x = origin.x + (pr->scan_step.horizontal * re) + pr->scan_size.width / 2;
  } else {
    mask->vertex[0].x = 0;
    mask->vertex[1].x = s.width - 1;
  }
  if (pr->scan_direction.vertical) {
    int32_t te = (int32_t)detect_edge(im, origin, (UphipDelta){0, -pr->scan_step.vertical},
                                      pr->scan_size.height, pr->scan_depth.vertical,
                                      pr->scan_threshold.vertical);
    int32_t be = (int32_t)detect_edge(im, origin, (UphipDelta){0, pr->scan_step.vertical},
                                      pr->scan_size.height, pr->scan_depth.vertical,
                                      pr->scan_threshold.vertical);
    mask->vertex[0].y = origin.y - (pr->scan_step.vertical * te) - pr->scan_size.height / 2;
    mask->vertex[1].y = origin.y + (pr->scan_step.vertical * be) + pr->scan_size.height / 2;
  } else {
    mask->vertex[0].y = 0;
    mask->vertex[1].y = s.height - 1;
  }
  UphipRectangleSize ms = rect_size(*mask);
  bool ok = true;
  if ((pr->minimum_width != -1 && ms.width < pr->minimum_width) ||
      (pr->maximum_width != -1 && ms.width > pr->maximum_width)) {
    mask->vertex[0].x = origin.x - pr->maximum_width / 2;
    mask->vertex[1].x = origin.x + pr->maximum_width / 2;
    ok = false;
  }
  if ((pr->minimum_height != -1 && ms.height < pr->minimum_height) ||
      (pr->maximum_height != -1 && ms.height > pr->maximum_height)) {
    mask->vertex[0].y = origin.y - pr->maximum_height / 2;
    mask->vertex[1].y = origin.y + pr->maximum_height / 2;
    ok = false;
  }
  return ok;
}

size_t o_detect_masks(OImage im, const UphipMaskDetectionParameters *pr,
                      const UphipPoint *points, size_t n, UphipRectangle *masks) {
  /* detect_masks_cpu, masks.c:181-209 */
  size_t count = 0;
  if (!pr->scan_direction.horizontal && !pr->scan_direction.vertical) return 0;
  for (size_t i = 0; i < n; i++) {
    detect_mask(im, pr, points[i], &masks[i]);
    const UphipRectangle inv = {{{-1, -1}, {-1, -1}}};
    if (memcmp(&masks[i], &inv, sizeof(inv)) != 0) count++;
  }
  return count;
}

void o_center_mask(OImage im, UphipPoint center, UphipRectangle area) {
  /* center_mask, masks.c:222-249 */
  const UphipRectangleSize s = rect_size(area);
  const UphipRectangle ia = full_image(im);
  const UphipPoint t = {center.x - s.width / 2, center.y - s.height / 2};
  UphipRectangle na = rect_from_size(t, s);
  if (point_in(na.vertex[0], ia) && point_in(na.vertex[1], ia)) {
    OImage n = create_compatible(im, s, true);
    o_copy_rectangle(im, n, area, (UphipPoint){0, 0});
    o_wipe_rectangle(im, area, im.background);
    o_copy_rectangle(n, im, full_image(n), t);
    o_free_image(&n);
  }
}

void o_align_mask(OImage im, UphipRectangle inside, UphipRectangle outside,
                  UphipMaskAlignmentParameters pr) {
  /* align_mask_cpu, masks.c:265-300 */
  const UphipRectangleSize is = rect_size(inside);
  UphipPoint t;
  if (pr.alignment.left)
    t.x = outside.vertex[0].x + pr.margin.horizontal;
  else if (pr.alignment.right)
    t.x = outside.vertex[1].x - is.width - pr.margin.horizontal;
  else
    t.x = (outside.vertex[0].x + outside.vertex[1].x - is.width) / 2;
  if (pr.alignment.top)
    t.y = outside.vertex[0].y + pr.margin.vertical;
  else if (pr.alignment.bottom)
    t.y = outside.vertex[1].y - is.height - pr.margin.vertical;
  else
    t.y = (outside.vertex[0].y + outside.vertex[1].y - is.height) / 2;
  OImage n = create_compatible(im, is, true);
  o_copy_rectangle(im, n, inside, (UphipPoint){0, 0});
  o_wipe_rectangle(im, inside, im.background);
  o_copy_rectangle(n, im, full_image(n), t);
  o_free_image(&n);
}

void o_apply_masks(OImage im, const UphipRectangle *masks, size_t count,
                   UphipPixel color) {
  /* apply_masks_cpu, masks.c:306-322 */
  if (count <= 0) return;
  for (int32_t y = 0; y < im.height; y++)
    for (int32_t x = 0; x < im.width; x++) {
      UphipPoint p = {x, y};
      bool inside = false;
      for (size_t n = 0; n < count && !inside; n++) inside = point_in(p, masks[n]);
      if (!inside) o_set_pixel(im, p, color);
    }
}

void o_apply_wipes(OImage im, const UphipWipes *w, UphipPixel color) {
  /* apply_wipes_cpu, masks.c:333-345 (rectangles not clipped: set_pixel drops) */
  for (size_t i = 0; i < w->count; i++) {
    UphipRectangle a = w->areas[i];
    for (int32_t y = a.vertex[0].y; y <= a.vertex[1].y; y++)
      for (int32_t x = a.vertex[0].x; x <= a.vertex[1].x; x++)
        o_set_pixel(im, (UphipPoint){x, y}, color);
  }
}

static UphipRectangle border_to_mask(OImage im, UphipBorder b) {
  /* border_to_mask, masks.c:351-366 */
  UphipRectangle m = {{{b.left, b.top},
                       {im.width - b.right - 1, im.height - b.bottom - 1}}};
  return m;
}

void o_apply_border(OImage im, UphipBorder b, UphipPixel color) {
  /* apply_border_cpu, masks.c:372-383 */
  if (b.left == 0 && b.top == 0 && b.right == 0 && b.bottom == 0) return;
  UphipRectangle m = border_to_mask(im, b);
  o_apply_masks(im, &m, 1, color);
}

static uint32_t detect_border_edge(OImage im, UphipRectangle outside, UphipDelta step,
                                   int32_t size, int32_t threshold) {
  /* detect_border_edge, masks.c:410-449 */
  UphipRectangle a = outside;
  UphipRectangleSize ms = rect_size(outside);
  int32_t max_step;
  if (step.vertical == 0) {
    if (step.horizontal > 0)
      a.vertex[1].x = outside.vertex[0].x + size;
    else
      a.vertex[0].x = outside.vertex[1].x - size;
    max_step = ms.width;
  } else {
    if (step.vertical > 0)
      a.vertex[1].y = outside.vertex[0].y + size;
    else
      a.vertex[0].y = outside.vertex[1].y - size;
    max_step = ms.height;
  }
  uint32_t result = 0;
  while (result < (uint32_t)max_step) {
    uint32_t cnt = (uint32_t)count_within_brightness(im, a, 0, im.abs_black_threshold, false);
    if (cnt >= (uint32_t)threshold) return result;
    a = rect_shift(a, step);
    result += (uint32_t)abs(step.horizontal + step.vertical);
  }
  return 0;
}

UphipBorder o_detect_border(OImage im, UphipBorderScanParameters pr,
                            UphipRectangle outside) {
  /* detect_border_cpu, masks.c:455-488 */
  UphipBorder b = {outside.vertex[0].x, outside.vertex[0].y,
                   im.width - outside.vertex[1].x, im.height - outside.vertex[1].y};
  if (pr.scan_direction.horizontal) {
    b.left += (int32_t)detect_border_edge(im, outside, (UphipDelta){pr.scan_step.horizontal, 0},
                                          pr.scan_size.width, pr.scan_threshold.horizontal);
    b.right += (int32_t)detect_border_edge(im, outside, (UphipDelta){-pr.scan_step.horizontal, 0},
                                           pr.scan_size.width, pr.scan_threshold.horizontal);
  }
  if (pr.scan_direction.vertical) {
    b.top += (int32_t)detect_border_edge(im, outside, (UphipDelta){0, pr.scan_step.vertical},
                                         pr.scan_size.height, pr.scan_threshold.vertical);
    b.bottom += (int32_t)detect_border_edge(im, outside, (UphipDelta){0, -pr.scan_step.vertical},
                                            pr.scan_size.height, pr.scan_threshold.vertical);
  }
  return b;
}

/* ------------------------------------------------------------------------
 * deskew.c
 * ---------------------------------------------------------------------- */
#define MAX_ROTATION_SCAN_SIZE 10000 /* deskew.c:18 */

static int edge_rotation_peak(OImage im, UphipRectangle mask,
                              const UphipDeskewParameters *pr, UphipDelta shift,
                              float m) {
  /* detect_edge_rotation_peak, deskew.c:48-146 */
  UphipRectangleSize size = rect_size(mask);
  int mid, half, side, outer, maxDepth, dep;
  float X, Y, sx, sy;
  int last = 0, diff = 0, maxDiff = 0, accumulated = 0;
  int maxBlacknessAbs = (int)(255 * pr->deskewScanSize * pr->deskewScanDepth);
  int scan = pr->deskewScanSize;
  if (shift.vertical == 0) {
    if (scan == -1) scan = size.height;
    scan = OMIN(OMIN(scan, MAX_ROTATION_SCAN_SIZE), size.height);
    maxDepth = size.width / 2;
    half = scan / 2;
    outer = (int)(fabsf(m) * half);
    mid = size.height / 2;
    side = shift.horizontal > 0 ? mask.vertex[0].x - outer : mask.vertex[1].x + outer;
    X = side + half * m;
    Y = mask.vertex[0].y + mid - half;
    sx = -m;
    sy = 1.0;
  } else {
    if (scan == -1) scan = size.width;
    scan = OMIN(OMIN(scan, MAX_ROTATION_SCAN_SIZE), size.width);
    maxDepth = size.height / 2;
    half = scan / 2;
    outer = (int)(fabsf(m) * half);
    mid = size.width / 2;
    side = shift.vertical > 0 ? mask.vertex[0].x - outer : mask.vertex[1].x + outer;
    X = mask.vertex[0].x + mid - half;
    Y = side - (half * m);
    sx = 1.0;
    sy = -m;
  }
  if (scan <= 0) return 0;
  UphipPoint *p = (UphipPoint *)malloc(sizeof(UphipPoint) * (size_t)scan);
  for (int i = 0; i < scan; i++) {
    p[i].x = (int)X;
    p[i].y = (int)Y;
    X += sx;
    Y += sy;
  }
  for (dep = 0; accumulated < maxBlacknessAbs && dep < maxDepth; dep++) {
    int blackness = 0;
    for (int i = 0; i < scan; i++) {
      UphipPoint pt = p[i];
      p[i].x += shift.horizontal;
      p[i].y += shift.vertical;
      if (point_in(pt, mask)) blackness += 255 - get_darkness_inverse(im, pt);
    }
    diff = blackness - last;
    last = blackness;
    if (diff >= maxDiff) maxDiff = diff;
    accumulated += blackness;
  }
  free(p);
  return dep < maxDepth ? maxDiff : 0;
}

static float edge_rotation(OImage im, UphipRectangle mask,
                           const UphipDeskewParameters *pr, UphipDelta shift) {
  /* detect_edge_rotation, deskew.c:153-174 */
  int max_peak = 0;
  float detected = 0.0;
  for (float r = 0.0; r <= pr->deskewScanRangeRad;
       r = (r >= 0.0) ? -(r + pr->deskewScanStepRad) : -r) {
    float m = tanf(r);
    int peak = edge_rotation_peak(im, mask, pr, shift, m);
    if (peak > max_peak) {
      detected = r;
      max_peak = peak;
    }
  }
  return detected;
}

int o_rotation_peaks(OImage im, UphipRectangle mask, const UphipDeskewParameters *pr,
                     int32_t *out, int capacity) {
  /* every peak detect_edge_rotation compares (deskew.c:153-174), edges in
   * detect_rotation_cpu's order (deskew.c:181-218) */
  const UphipDelta shifts[4] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}};
  const bool on[4] = {pr->scan_edges.left, pr->scan_edges.top, pr->scan_edges.right,
                      pr->scan_edges.bottom};
  int n = 0;
  for (int k = 0; k < 4; k++) {
    if (!on[k]) continue;
    for (float r = 0.0; r <= pr->deskewScanRangeRad;
         r = (r >= 0.0) ? -(r + pr->deskewScanStepRad) : -r) {
      if (n >= capacity) return -1;
      out[n++] = edge_rotation_peak(im, mask, pr, shifts[k], tanf(r));
    }
  }
  return n;
}

float o_detect_rotation(OImage im, UphipRectangle mask,
                        const UphipDeskewParameters *pr) {
  /* detect_rotation_cpu, deskew.c:181-241 */
  float rot[4];
  int count = 0;
  if (pr->scan_edges.left) rot[count++] = edge_rotation(im, mask, pr, (UphipDelta){1, 0});
  if (pr->scan_edges.top) rot[count++] = -edge_rotation(im, mask, pr, (UphipDelta){0, 1});
  if (pr->scan_edges.right) rot[count++] = edge_rotation(im, mask, pr, (UphipDelta){-1, 0});
  if (pr->scan_edges.bottom) rot[count++] = -edge_rotation(im, mask, pr, (UphipDelta){0, -1});
  float total = 0.0;
  for (int i = 0; i < count; i++) total += rot[i];
  float average = total / count;
  total = 0.0;
  /* called through a pointer: the reference's default (-O0) build calls
   * glibc powf, which gcc -O2 would otherwise fold into x*x */
  static float (*volatile pw)(float, float) = powf;
  for (int i = 0; i < count; i++) total += pw(rot[i] - average, 2);
  float deviation = sqrtf(total);
  return deviation <= pr->deskewScanDeviationRad ? average : 0.0f;
}

static void rotate_into(OImage src, UphipRectangle sa, OImage dst, const float radians,
                        int32_t interp) {
  /* rotate, deskew.c:248-270 */
  UphipRectangle ta = full_image(dst);
  UphipRectangle na = rect_normalize(sa);
  UphipRectangleSize ss = rect_size(na), ts = rect_size(ta);
  const float scx = na.vertex[0].x + ss.width / 2.0f;
  const float scy = na.vertex[0].y + ss.height / 2.0f;
  const float tcx = ta.vertex[0].x + ts.width / 2.0f;
  const float tcy = ta.vertex[0].y + ts.height / 2.0f;
  const float sinval = sinf(radians);
  const float cosval = cosf(radians);
  for (int32_t y = ta.vertex[0].y; y <= ta.vertex[1].y; y++)
    for (int32_t x = ta.vertex[0].x; x <= ta.vertex[1].x; x++) {
      const float srcX = scx + (x - tcx) * cosval + (y - tcy) * sinval;
      const float srcY = scy + (y - tcy) * cosval - (x - tcx) * sinval;
      o_set_pixel(dst, (UphipPoint){x, y}, interpolate(src, srcX, srcY, interp));
    }
}

void o_deskew(OImage src, UphipRectangle mask, float radians, int32_t interp) {
  /* deskew_cpu, deskew.c:272-286 */
  OImage r = create_compatible(src, rect_size(mask), true);
  rotate_into(src, mask, r, -radians, interp);
  o_copy_rectangle(r, src, full_image(r), mask.vertex[0]);
  o_free_image(&r);
}

/* ------------------------------------------------------------------------
 * Sheet pipeline — src/core/sheet_stages.c for a fresh SheetProcessState
 * (sheet_process.c:29-84: mask_count = 0, previous_size = {-1,-1}).
 * ---------------------------------------------------------------------- */
#define DIS(o, bit) (((o)->disable & (bit)) != 0)

int o_process_sheet(const UphipOptions *o, const OImage *pages, OImage *sheet_out,
                    int32_t *out_format, OReport *rep) {
  UphipRectangleSize input_size = {-1, -1};
  OImage sheet = {0};
  int32_t out_fmt = o->output_pixel_format;
  memset(rep, 0, sizeof(*rep));

  /* sheet_stage_decode, sheet_stages.c:44-185 */
  for (int j = 0; j < o->input_count; j++) {
    OImage page = {0};
    bool have = pages[j].data != NULL;
    if (have) {
      page = o_create_image((UphipRectangleSize){pages[j].width, pages[j].height},
                            pages[j].format, false, o->sheet_background,
                            o->abs_black_threshold);
      for (int32_t y = 0; y < page.height; y++)
        memcpy(page.data + y * page.linesize, pages[j].data + y * pages[j].linesize,
               (size_t)o_min_linesize(page.width, page.format));
      if (out_fmt == UPHIP_FMT_NONE) out_fmt = page.format;
      if (o->pre_rotate != 0) o_flip_rotate_90(&page, o->pre_rotate / 90);
      UphipRectangleSize iss = {page.width * o->input_count, page.height};
      input_size = coerce_size(input_size, coerce_size(o->sheet_size, iss));
    }
    if (sheet.data == NULL && input_size.width != -1 && input_size.height != -1)
      sheet = o_create_image(input_size, UPHIP_FMT_RGB24, true, o->sheet_background,
                             o->abs_black_threshold);
    if (have) {
      o_center_image(page, sheet, (UphipPoint){input_size.width * j / o->input_count, 0},
                     (UphipRectangleSize){input_size.width / o->input_count,
                                          input_size.height});
      o_free_image(&page);
    }
  }
  if (sheet.data == NULL) return -1; /* sheet size unknown (fresh job) */

  /* sheet_stage_pre, sheet_stages.c:187-325 */
  if (o->pre_mirror.horizontal || o->pre_mirror.vertical) o_mirror(sheet, o->pre_mirror);
  if (o->pre_shift.horizontal != 0 || o->pre_shift.vertical != 0)
    o_shift_image(&sheet, o->pre_shift);
  if (o->pre_mask_count > 0)
    o_apply_masks(sheet, o->pre_masks, o->pre_mask_count, o->mask_color);
  input_size = coerce_size(o->stretch_size, image_size(sheet));
  input_size.width *= o->pre_zoom_factor;
  input_size.height *= o->pre_zoom_factor;
  o_stretch_and_replace(&sheet, input_size, o->interpolate_type);
  if (o->page_size.width != -1 || o->page_size.height != -1) {
    input_size = coerce_size(o->page_size, image_size(sheet));
    o_resize_and_replace(&sheet, input_size, o->interpolate_type);
  }

  UphipPoint points[UPHIP_MAX_POINTS];
  size_t point_count = o->point_count;
  memcpy(points, o->points, sizeof(UphipPoint) * point_count);
  int32_t mask_max_w = o->mask_detection_parameters.maximum_width;
  int32_t mask_max_h = o->mask_detection_parameters.maximum_height;
  UphipRectangle outside[UPHIP_MAX_PAGES];
  size_t outside_count = 0;
  const int32_t W = sheet.width, H = sheet.height;
  if (o->layout == UPHIP_LAYOUT_SINGLE) {
    if (point_count == 0) points[point_count++] = (UphipPoint){W / 2, H / 2};
    if (mask_max_w == -1) mask_max_w = W;
    if (mask_max_h == -1) mask_max_h = H;
    if (outside_count == 0) outside[outside_count++] = full_image(sheet);
  } else if (o->layout == UPHIP_LAYOUT_DOUBLE) {
    if (point_count == 0) {
      points[point_count++] = (UphipPoint){W / 4, H / 2};
      points[point_count++] = (UphipPoint){W - W / 4, H / 2};
    }
    if (mask_max_w == -1) mask_max_w = W / 2;
    if (mask_max_h == -1) mask_max_h = H;
    if (outside_count == 0) {
      outside[outside_count++] = (UphipRectangle){{{0, 0}, {W / 2, H - 1}}};
      outside[outside_count++] = (UphipRectangle){{{W / 2, 0}, {W - 1, H - 1}}};
    }
  }
  if (mask_max_w == -1) mask_max_w = W;
  if (mask_max_h == -1) mask_max_h = H;
  if (!DIS(o, UPHIP_NO_WIPE)) o_apply_wipes(sheet, &o->pre_wipes, o->mask_color);
  if (!DIS(o, UPHIP_NO_BORDER)) o_apply_border(sheet, o->pre_border, o->mask_color);

  UphipMaskDetectionParameters mp = o->mask_detection_parameters;
  mp.maximum_width = mask_max_w;
  mp.maximum_height = mask_max_h;
  UphipBlackfilterParameters bp = o->blackfilter_parameters;
  if (bp.exclusions_count == 0 && o->layout != UPHIP_LAYOUT_NONE) {
    if (o->layout == UPHIP_LAYOUT_SINGLE) {
      bp.exclusions[bp.exclusions_count++] =
          rect_from_size((UphipPoint){W / 4, H / 4}, (UphipRectangleSize){W / 2, H / 2});
    } else if (o->layout == UPHIP_LAYOUT_DOUBLE) {
      UphipRectangleSize fs = {W / 4, H / 2};
      UphipPoint f1 = {W / 8, H / 4};
      UphipPoint f2 = {f1.x + W / 2, f1.y};
      bp.exclusions[bp.exclusions_count++] = rect_from_size(f1, fs);
      bp.exclusions[bp.exclusions_count++] = rect_from_size(f2, fs);
    }
  }

  /* sheet_stage_filters, sheet_stages.c:327-357 */
  if (!DIS(o, UPHIP_NO_BLACKFILTER)) o_blackfilter(sheet, &bp);
  if (!DIS(o, UPHIP_NO_NOISEFILTER))
    o_noisefilter(sheet, o->noisefilter_intensity, o->abs_white_threshold);
  if (!DIS(o, UPHIP_NO_BLURFILTER))
    o_blurfilter(sheet, o->blurfilter_parameters, o->abs_white_threshold);

  /* sheet_stage_masks, sheet_stages.c:359-386: the first detection's count is
   * discarded (mask_count stays 0 for a fresh job) */
  UphipRectangle masks[UPHIP_MAX_POINTS];
  size_t mask_count = 0;
  memset(masks, 0, sizeof(masks));
  if (!DIS(o, UPHIP_NO_MASK_SCAN)) o_detect_masks(sheet, &mp, points, point_count, masks);
  if (mask_count > 0) o_apply_masks(sheet, masks, mask_count, o->mask_color);
  if (!DIS(o, UPHIP_NO_GRAYFILTER)) o_grayfilter(sheet, o->grayfilter_parameters);

  /* sheet_stage_deskew, sheet_stages.c:388-413 */
  if (!DIS(o, UPHIP_NO_DESKEW)) {
    if (!DIS(o, UPHIP_NO_MASK_SCAN))
      mask_count = o_detect_masks(sheet, &mp, points, point_count, masks);
    for (size_t i = 0; i < mask_count; i++) {
      float r = o_detect_rotation(sheet, masks[i], &o->deskew_parameters);
      if (i < UPHIP_MAX_PAGES) rep->rotation[i] = r;
      if (r != 0.0) o_deskew(sheet, masks[i], r, o->interpolate_type);
    }
  }

  /* sheet_stage_post, sheet_stages.c:415-534 */
  if (!DIS(o, UPHIP_NO_MASK_CENTER)) {
    if (!DIS(o, UPHIP_NO_MASK_SCAN))
      mask_count = o_detect_masks(sheet, &mp, points, point_count, masks);
    for (size_t i = 0; i < mask_count; i++) o_center_mask(sheet, points[i], masks[i]);
  }
  rep->mask_count = (int32_t)mask_count;
  for (size_t i = 0; i < mask_count && i < UPHIP_MAX_PAGES; i++) rep->masks[i] = masks[i];
  if (!DIS(o, UPHIP_NO_WIPE)) {
    UphipWipes w = o->wipes;
    if (o->layout == UPHIP_LAYOUT_DOUBLE && (o->middle_wipe[0] > 0 || o->middle_wipe[1] > 0))
      w.areas[w.count++] = (UphipRectangle){{{W / 2 - o->middle_wipe[0], 0},
                                             {W / 2 + o->middle_wipe[1], H - 1}}};
    o_apply_wipes(sheet, &w, o->mask_color);
  }
  if (!DIS(o, UPHIP_NO_BORDER)) o_apply_border(sheet, o->border, o->mask_color);
  if (!DIS(o, UPHIP_NO_BORDER_SCAN)) {
    UphipRectangle abm[UPHIP_MAX_PAGES];
    for (size_t i = 0; i < outside_count; i++)
      abm[i] = border_to_mask(sheet, o_detect_border(sheet, o->border_scan_parameters,
                                                     outside[i]));
    o_apply_masks(sheet, abm, outside_count, o->mask_color);
    for (size_t i = 0; i < outside_count; i++) {
      rep->border_masks[i] = abm[i];
      if (!DIS(o, UPHIP_NO_BORDER_ALIGN))
        o_align_mask(sheet, abm[i], outside[i], o->mask_alignment_parameters);
    }
  }
  if (!DIS(o, UPHIP_NO_WIPE)) o_apply_wipes(sheet, &o->post_wipes, o->mask_color);
  if (!DIS(o, UPHIP_NO_BORDER)) o_apply_border(sheet, o->post_border, o->mask_color);
  if (o->post_mirror.horizontal || o->post_mirror.vertical) o_mirror(sheet, o->post_mirror);
  if (o->post_shift.horizontal != 0 || o->post_shift.vertical != 0)
    o_shift_image(&sheet, o->post_shift);
  if (o->post_rotate != 0) o_flip_rotate_90(&sheet, o->post_rotate / 90);
  input_size = coerce_size(o->post_stretch_size, image_size(sheet));
  input_size.width *= o->post_zoom_factor;
  input_size.height *= o->post_zoom_factor;
  o_stretch_and_replace(&sheet, input_size, o->interpolate_type);
  if (o->post_page_size.width != -1 || o->post_page_size.height != -1) {
    input_size = coerce_size(o->post_page_size, image_size(sheet));
    o_resize_and_replace(&sheet, input_size, o->interpolate_type);
  }

  /* sheet_stage_output, sheet_stages.c:536-552 */
  if (out_fmt == UPHIP_FMT_NONE) out_fmt = sheet.format;
  *out_format = out_fmt;
  rep->width = sheet.width;
  rep->height = sheet.height;
  *sheet_out = sheet;
  return 0;
}

OImage o_convert_for_save(OImage in, int32_t fmt) {
  /* saveImage, file.c:187-259 */
  if (fmt == UPHIP_FMT_Y400A) fmt = UPHIP_FMT_GRAY8;
  if (fmt == UPHIP_FMT_MONOBLACK) fmt = UPHIP_FMT_MONOWHITE;
  OImage out = o_create_image((UphipRectangleSize){in.width, in.height}, fmt, false,
                              in.background, in.abs_black_threshold);
  if (in.format == fmt) {
    for (int32_t y = 0; y < in.height; y++)
      memcpy(out.data + y * out.linesize, in.data + y * in.linesize,
             (size_t)o_min_linesize(in.width, fmt));
    return out;
  }
  if (fmt == UPHIP_FMT_MONOWHITE &&
      (in.format == UPHIP_FMT_RGB24 || in.format == UPHIP_FMT_GRAY8)) {
    /* fast paths file.c:209-238: bit set when gray < abs_black_threshold */
    for (int32_t y = 0; y < in.height; y++) {
      uint8_t *d = out.data + y * out.linesize;
      for (int32_t x = 0; x < in.width; x++) {
        int g = get_gray(in, (UphipPoint){x, y});
        if (x % 8 == 0) d[x / 8] = 0;
        if (g < in.abs_black_threshold) d[x / 8] |= (uint8_t)(0x80 >> (x % 8));
      }
    }
    return out;
  }
  o_copy_rectangle(in, out, full_image(in), (UphipPoint){0, 0});
  return out;
}

/* ------------------------------------------------------------------------
 * Defaults — lib/options.c:23-173 (options_init + options_init_filter_defaults)
 * and the CLI-derived values of src/cli/cli_options.c:229-269,1108-1109.
 * ---------------------------------------------------------------------- */
static float deg2rad(float d) { return d * M_PI / 180.0; } /* deskew.c:20 */

void o_options_init(UphipOptions *o) {
  memset(o, 0, sizeof(*o));
  o->layout = UPHIP_LAYOUT_SINGLE;
  o->input_count = 1;
  o->output_count = 1;
  o->output_pixel_format = UPHIP_FMT_NONE;
  o->sheet_size = o->page_size = o->post_page_size = (UphipRectangleSize){-1, -1};
  o->stretch_size = o->post_stretch_size = (UphipRectangleSize){-1, -1};
  o->pre_zoom_factor = 1.0;
  o->post_zoom_factor = 1.0;
  o->sheet_background = PX_WHITE;
  o->mask_color = PX_WHITE;
  float blackThreshold = 0.33, whiteThreshold = 0.9;
  o->abs_black_threshold = (uint8_t)(0xFF * (1.0 - blackThreshold));
  o->abs_white_threshold = (uint8_t)(0xFF * (whiteThreshold));
  o->interpolate_type = UPHIP_INTERP_CUBIC;
  o->noisefilter_intensity = 4;

  UphipBlackfilterParameters *bf = &o->blackfilter_parameters;
  bf->scan_size = (UphipRectangleSize){20, 20};
  bf->scan_step = (UphipDelta){5, 5};
  bf->scan_depth.horizontal = 500;
  bf->scan_depth.vertical = 500;
  bf->scan_direction = (UphipDirection){true, true};
  bf->abs_threshold = (uint8_t)(UINT8_MAX * 0.95f);
  bf->intensity = 20;
  o->blurfilter_parameters =
      (UphipBlurfilterParameters){{100, 100}, {50, 50}, 0.01f};
  o->grayfilter_parameters.scan_size = (UphipRectangleSize){50, 50};
  o->grayfilter_parameters.scan_step = (UphipDelta){20, 20};
  o->grayfilter_parameters.abs_threshold = (uint8_t)(UINT8_MAX * 0.5f);

  UphipDeskewParameters *dp = &o->deskew_parameters;
  dp->deskewScanRangeRad = deg2rad(5.0f);
  dp->deskewScanStepRad = deg2rad(0.1f);
  dp->deskewScanDeviationRad = deg2rad(1.0f);
  dp->deskewScanSize = 1500;
  dp->deskewScanDepth = 0.5f;
  dp->scan_edges = (UphipEdges){true, false, true, false};

  UphipMaskDetectionParameters *mp = &o->mask_detection_parameters;
  mp->scan_size = (UphipRectangleSize){50, 50};
  mp->scan_step = (UphipDelta){5, 5};
  mp->scan_depth.horizontal = -1;
  mp->scan_depth.vertical = -1;
  mp->scan_direction = (UphipDirection){true, false};
  mp->scan_threshold.horizontal = 0.1f;
  mp->scan_threshold.vertical = 0.1f;
  mp->minimum_width = 100;
  mp->minimum_height = 100;
  mp->maximum_width = -1;
  mp->maximum_height = -1;

  UphipBorderScanParameters *bs = &o->border_scan_parameters;
  bs->scan_size = (UphipRectangleSize){5, 5};
  bs->scan_step = (UphipDelta){5, 5};
  bs->scan_threshold.horizontal = 5;
  bs->scan_threshold.vertical = 5;
  bs->scan_direction = (UphipDirection){false, true};
}

size_t oracle_abi_sizeof(const char *name) {
#define S(T) if (!strcmp(name, #T)) return sizeof(T);
  S(UphipPoint) S(UphipDelta) S(UphipDirection) S(UphipEdges) S(UphipPixel)
  S(UphipRectangle) S(UphipRectangleSize) S(UphipBorder) S(UphipWipes)
  S(UphipBlackfilterParameters) S(UphipBlurfilterParameters)
  S(UphipGrayfilterParameters) S(UphipMaskDetectionParameters)
  S(UphipMaskAlignmentParameters) S(UphipBorderScanParameters)
  S(UphipDeskewParameters) S(UphipOptions) S(UphipSheetReport) S(UphipBatchGeometry)
#undef S
  return 0;
}
