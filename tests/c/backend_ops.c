/* backend_ops.c — the 20 ImageBackend ops called from C through the HIP
 * backend's vtable (uphip_backend(), the image_backend_get() peer of
 * imageprocess/backend.c:135-157), each compared byte for byte with the
 * oracle (oracle/oracle.c, the CPU restatement) on the same input, in all five
 * pixel formats.  This is what the reference's own C callers (sheet_stages.c,
 * image_pipeline.c) would do after `image_backend_select(UNPAPER_DEVICE_HIP)`.
 *
 * TEST INFRASTRUCTURE (links the oracle); run by tests/test_c_abi_gpu.py on a
 * GPU box.  Exit status 0 = every check equal.  Build: `make ctest`.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/unpaper_hip.h"
#include "../../oracle/oracle.h"
#include "pages.h"

static int g_checks, g_failures;
static const UphipBackend *B;

#define W0 620
#define H0 877

static const char *fmt_name(int f) {
  static const char *n[] = {"GRAY8", "Y400A", "RGB24", "MONOWHITE", "MONOBLACK"};
  return f >= 0 && f < 5 ? n[f] : "?";
}

static void fail_check(const char *op, int fmt, const char *what) {
  g_failures++;
  fprintf(stderr, "MISMATCH %s [%s]: %s\n", op, fmt_name(fmt), what);
}

static void api_error(const char *op) {
  const char *e = uphip_last_error();
  if (e) {
    fprintf(stderr, "ERROR %s: %s\n", op, e);
    g_failures++;
    uphip_clear_error();
  }
}

static UphipImage upload(OImage h) {
  UphipImage d = uphip_create_image((UphipRectangleSize){h.width, h.height}, h.format, false,
                                    h.background, h.abs_black_threshold);
  uphip_image_upload(d, h.data, h.linesize);
  api_error("upload");
  return d;
}

/* exact comparison of the visible pixels */
static void compare(const char *op, OImage h, UphipImage d) {
  g_checks++;
  const UphipRectangleSize s = uphip_size_of_image(d);
  const int fmt = uphip_image_format(d);
  char msg[256];
  if (s.width != h.width || s.height != h.height || fmt != h.format) {
    snprintf(msg, sizeof msg, "geometry %dx%d/%d vs %dx%d/%d", s.width, s.height, fmt, h.width,
             h.height, h.format);
    fail_check(op, h.format, msg);
    return;
  }
  uint8_t *buf = malloc((size_t)h.linesize * h.height);
  uphip_image_download(d, buf, h.linesize);
  api_error("download");
  const bool mono = fmt == UPHIP_FMT_MONOWHITE || fmt == UPHIP_FMT_MONOBLACK;
  const int64_t rb = mono ? 0 : o_min_linesize(h.width, fmt);
  for (int y = 0; y < h.height; y++) {
    const uint8_t *a = h.data + (int64_t)y * h.linesize, *b = buf + (int64_t)y * h.linesize;
    if (mono) {
      for (int x = 0; x < h.width; x++)
        if (((a[x >> 3] ^ b[x >> 3]) >> (7 - (x & 7))) & 1) {
          snprintf(msg, sizeof msg, "pixel (%d,%d)", x, y);
          fail_check(op, fmt, msg);
          free(buf);
          return;
        }
    } else if (memcmp(a, b, (size_t)rb)) {
      int x = 0;
      while (a[x] == b[x]) x++;
      snprintf(msg, sizeof msg, "byte %d of row %d: %d vs %d", x, y, a[x], b[x]);
      fail_check(op, fmt, msg);
      free(buf);
      return;
    }
  }
  free(buf);
}

static void check_int(const char *op, int fmt, long long a, long long b, const char *what) {
  g_checks++;
  if (a != b) {
    char msg[160];
    snprintf(msg, sizeof msg, "%s: %lld (oracle) vs %lld (hip)", what, a, b);
    fail_check(op, fmt, msg);
  }
}

static UphipRectangle rect(int x0, int y0, int x1, int y1) {
  return (UphipRectangle){{{x0, y0}, {x1, y1}}};
}

static void run_format(int fmt, const UphipOptions *o) {
  const UphipPixel red = {200, 30, 40}, black = {0, 0, 0};
  const UphipPixel color = fmt == UPHIP_FMT_RGB24 ? red : black;
  uint32_t seed = 3;  /* page 3: the dark band (blackfilter flood fill) */
#define FRESH(h, d) OImage h = host_page(fmt, W0, H0, seed); UphipImage d = upload(h)
#define DONE(h, d) do { o_free_image(&h); uphip_free_image(&d); } while (0)
  { /* 1 wipe_rectangle */
    FRESH(h, d);
    o_wipe_rectangle(h, rect(10, 20, 200, 150), color);
    B->wipe_rectangle(d, rect(10, 20, 200, 150), color);
    api_error("wipe_rectangle");
    compare("wipe_rectangle", h, d);
    DONE(h, d);
  }
  { /* 2 copy_rectangle, 3 center_image */
    FRESH(h, d);
    OImage ht = o_create_image((UphipRectangleSize){W0 - 100, H0 - 50}, fmt, true, h.background,
                               170);
    UphipImage dt = uphip_create_image((UphipRectangleSize){W0 - 100, H0 - 50}, fmt, true,
                                       h.background, 170);
    o_copy_rectangle(h, ht, rect(30, 40, 400, 500), (UphipPoint){-5, 17});
    B->copy_rectangle(d, dt, rect(30, 40, 400, 500), (UphipPoint){-5, 17});
    api_error("copy_rectangle");
    compare("copy_rectangle", ht, dt);
    o_center_image(h, ht, (UphipPoint){0, 0}, (UphipRectangleSize){W0 - 100, H0 - 50});
    B->center_image(d, dt, (UphipPoint){0, 0}, (UphipRectangleSize){W0 - 100, H0 - 50});
    api_error("center_image");
    compare("center_image", ht, dt);
    o_free_image(&ht);
    uphip_free_image(&dt);
    DONE(h, d);
  }
  { /* 4 stretch_and_replace, 5 resize_and_replace */
    FRESH(h, d);
    o_stretch_and_replace(&h, (UphipRectangleSize){W0 * 3 / 4, H0 * 5 / 4}, UPHIP_INTERP_CUBIC);
    B->stretch_and_replace(&d, (UphipRectangleSize){W0 * 3 / 4, H0 * 5 / 4}, UPHIP_INTERP_CUBIC);
    api_error("stretch_and_replace");
    compare("stretch_and_replace", h, d);
    o_resize_and_replace(&h, (UphipRectangleSize){W0 + 37, H0 - 20}, UPHIP_INTERP_LINEAR);
    B->resize_and_replace(&d, (UphipRectangleSize){W0 + 37, H0 - 20}, UPHIP_INTERP_LINEAR);
    api_error("resize_and_replace");
    compare("resize_and_replace", h, d);
    DONE(h, d);
  }
  { /* 6 flip_rotate_90, 7 mirror, 8 shift_image */
    FRESH(h, d);
    o_flip_rotate_90(&h, 1);
    B->flip_rotate_90(&d, UPHIP_ROTATE_CLOCKWISE);
    api_error("flip_rotate_90");
    compare("flip_rotate_90", h, d);
    o_mirror(h, (UphipDirection){true, true});
    B->mirror(d, (UphipDirection){true, true});
    api_error("mirror");
    compare("mirror", h, d);
    o_shift_image(&h, (UphipDelta){13, -7});
    B->shift_image(&d, (UphipDelta){13, -7});
    api_error("shift_image");
    compare("shift_image", h, d);
    DONE(h, d);
  }
  { /* 9 apply_masks, 10 apply_wipes, 11 apply_border */
    FRESH(h, d);
    const UphipRectangle m[2] = {rect(100, 100, 500, 700), rect(-20, 650, 300, 900)};
    o_apply_masks(h, m, 2, color);
    B->apply_masks(d, m, 2, color);
    api_error("apply_masks");
    compare("apply_masks", h, d);
    UphipWipes wp;
    memset(&wp, 0, sizeof wp);
    wp.count = 2;
    wp.areas[0] = rect(0, 0, 50, 60);
    wp.areas[1] = rect(580, 800, 700, 900);
    o_apply_wipes(h, &wp, color);
    B->apply_wipes(d, wp, color);
    api_error("apply_wipes");
    compare("apply_wipes", h, d);
    o_apply_border(h, (UphipBorder){5, 6, 7, 8}, color);
    B->apply_border(d, (UphipBorder){5, 6, 7, 8}, color);
    api_error("apply_border");
    compare("apply_border", h, d);
    DONE(h, d);
  }
  { /* 12 detect_masks, 13 align_mask, 14 detect_border */
    FRESH(h, d);
    UphipMaskDetectionParameters mp = o->mask_detection_parameters;
    const UphipPoint pts[2] = {{W0 / 2, H0 / 2}, {W0 / 4, H0 / 3}};
    UphipRectangle mh[2], md[2];
    const size_t nh = o_detect_masks(h, &mp, pts, 2, mh);
    const size_t nd = B->detect_masks(d, mp, pts, 2, md);
    api_error("detect_masks");
    check_int("detect_masks", fmt, (long long)nh, (long long)nd, "count");
    for (int i = 0; i < 2; i++) {
      check_int("detect_masks", fmt, mh[i].vertex[0].x, md[i].vertex[0].x, "x0");
      check_int("detect_masks", fmt, mh[i].vertex[0].y, md[i].vertex[0].y, "y0");
      check_int("detect_masks", fmt, mh[i].vertex[1].x, md[i].vertex[1].x, "x1");
      check_int("detect_masks", fmt, mh[i].vertex[1].y, md[i].vertex[1].y, "y1");
    }
    const UphipMaskAlignmentParameters ap = {{true, true, false, false}, {10, 12}};
    o_align_mask(h, mh[0], rect(0, 0, W0 - 1, H0 - 1), ap);
    B->align_mask(d, mh[0], rect(0, 0, W0 - 1, H0 - 1), ap);
    api_error("align_mask");
    compare("align_mask", h, d);
    UphipBorderScanParameters bp = o->border_scan_parameters;
    bp.scan_direction = (UphipDirection){true, true};
    const UphipBorder bh = o_detect_border(h, bp, rect(0, 0, W0 - 1, H0 - 1));
    const UphipBorder bd = B->detect_border(d, bp, rect(0, 0, W0 - 1, H0 - 1));
    api_error("detect_border");
    check_int("detect_border", fmt, bh.left, bd.left, "left");
    check_int("detect_border", fmt, bh.top, bd.top, "top");
    check_int("detect_border", fmt, bh.right, bd.right, "right");
    check_int("detect_border", fmt, bh.bottom, bd.bottom, "bottom");
    DONE(h, d);
  }
  { /* 15 blackfilter, 16 noisefilter, 17 blurfilter, 18 grayfilter */
    FRESH(h, d);
    UphipBlackfilterParameters bf = o->blackfilter_parameters;
    o_blackfilter(h, &bf);
    B->blackfilter(d, bf);
    api_error("blackfilter");
    compare("blackfilter", h, d);
    o_noisefilter(h, o->noisefilter_intensity, o->abs_white_threshold);
    B->noisefilter(d, o->noisefilter_intensity, o->abs_white_threshold);
    api_error("noisefilter");
    compare("noisefilter", h, d);
    o_blurfilter(h, o->blurfilter_parameters, o->abs_white_threshold);
    B->blurfilter(d, o->blurfilter_parameters, o->abs_white_threshold);
    api_error("blurfilter");
    compare("blurfilter", h, d);
    o_grayfilter(h, o->grayfilter_parameters);
    B->grayfilter(d, o->grayfilter_parameters);
    api_error("grayfilter");
    compare("grayfilter", h, d);
    DONE(h, d);
  }
  { /* 19 detect_rotation, 20 deskew */
    seed = 5;
    FRESH(h, d);
    const UphipRectangle m = rect(60, 80, W0 - 61, H0 - 81);
    UphipDeskewParameters dp = o->deskew_parameters;
    const float rh = o_detect_rotation(h, m, &dp);
    const float rd = B->detect_rotation(d, m, dp);
    api_error("detect_rotation");
    uint32_t bh, bd;
    memcpy(&bh, &rh, 4);
    memcpy(&bd, &rd, 4);
    check_int("detect_rotation", fmt, bh, bd, "float bits");
    const float rad = rh != 0.0f ? rh : 0.0123f;
    o_deskew(h, m, rad, UPHIP_INTERP_CUBIC);
    B->deskew(d, m, rad, UPHIP_INTERP_CUBIC);
    api_error("deskew");
    compare("deskew", h, d);
    DONE(h, d);
  }
#undef FRESH
#undef DONE
}

int main(void) {
  const UphipInitStatus st = uphip_try_init();
  if (st != UPHIP_INIT_OK) {
    fprintf(stderr, "backend_ops: no HIP device (%s)\n", uphip_init_status_string(st));
    return 2;
  }
  B = uphip_backend();
  if (!B || !B->name) {
    fprintf(stderr, "backend_ops: no vtable\n");
    return 2;
  }
  UphipOptions o;
  uphip_options_init(&o);
  for (int fmt = UPHIP_FMT_GRAY8; fmt <= UPHIP_FMT_MONOBLACK; fmt++) run_format(fmt, &o);
  printf("backend_ops: backend \"%s\", 20 ops x 5 formats, %d checks, %d mismatches\n", B->name,
         g_checks, g_failures);
  return g_failures ? 1 : 0;
}
