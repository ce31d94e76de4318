/* adapter_main.c — the reference-side adapter (integration/backend_hip.c)
 * driven the way unpaper-gpu's stages drive a backend: the 20 ops on the
 * reference's own `Image` and value types (compiled against
 * the reference's imageprocess headers), each result brought back with
 * backend_hip_ensure_cpu() and compared byte for byte with the oracle in all
 * five pixel formats.  Host-side edits between ops go through
 * backend_hip_mark_cpu_dirty(), so the residency protocol is exercised too.
 *
 * The frame here is a plain struct standing in for AVFrame (FFmpeg headers
 * are not in this image): it implements the three hooks of
 * integration/hip_frame.h the way integration/backend_hip_av.c does with
 * libavutil.
 *
 * TEST INFRASTRUCTURE (links the oracle); built by `make adapter` when the
 * reference tree is present, run by tests/test_c_abi_gpu.py.  Exit 0 = every
 * check equal, 2 = no HIP device.
 */
#include <stdio.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include "backend_hip.h"
#include "pages.h"

/* ---- the frame hooks over a plain struct -------------------------------- */
struct AVFrame {
  int32_t width, height;
  UphipPixelFormat format;
  uint8_t *data;
  int64_t linesize;
  bool has_state;
  HipState st;
};

HipState *hip_state(AVFrame *f) {
  if (!f->has_state) {
    memset(&f->st, 0, sizeof f->st);
    f->st.host_newer = true;
    f->has_state = true;
  }
  return &f->st;
}

HipFrameView hip_frame_view(AVFrame *f) {
  return (HipFrameView){f->width, f->height, f->format, f->data, f->linesize};
}

static Image new_image(int32_t w, int32_t h, UphipPixelFormat fmt, Pixel bg, uint8_t thr) {
  AVFrame *f = calloc(1, sizeof *f);
  f->width = w;
  f->height = h;
  f->format = fmt;
  f->linesize = (o_min_linesize(w, fmt) + 31) & ~(int64_t)31; /* av_frame_get_buffer(.., 8)-like */
  f->data = calloc((size_t)(f->linesize * h), 1);
  return (Image){.frame = f, .background = bg, .abs_black_threshold = thr};
}

static void free_img(Image *im) {
  if (!im->frame) return;
  if (im->frame->has_state) backend_hip_release(&im->frame->st);
  free(im->frame->data);
  free(im->frame);
  im->frame = NULL;
}

void hip_adopt(Image *pImage, UphipImage d) {
  const UphipRectangleSize s = uphip_size_of_image(d);
  if (getenv("ADAPTER_TRACE")) fprintf(stderr, "  adopt %dx%d\n", s.width, s.height);
  Image n = new_image(s.width, s.height, pImage->frame->format, pImage->background,
                      pImage->abs_black_threshold);
  HipState *st = hip_state(n.frame);
  st->img = d;
  st->host_newer = false;
  st->device_newer = true;
  free_img(pImage);
  *pImage = n;
}

/* ---- checks --------------------------------------------------------------- */
static int g_checks, g_failures;

#define CP(T, v)                    \
  ({                                \
    T cp_;                          \
    _Static_assert(sizeof cp_ == sizeof(v), #T); \
    memcpy(&cp_, &(v), sizeof cp_); \
    cp_;                            \
  })

static const char *fmt_name(int f) {
  static const char *n[] = {"GRAY8", "Y400A", "RGB24", "MONOWHITE", "MONOBLACK"};
  return f >= 0 && f < 5 ? n[f] : "?";
}

static void api_error(const char *op) {
  const char *e = uphip_last_error();
  if (e) {
    fprintf(stderr, "ERROR %s: %s\n", op, e);
    g_failures++;
    uphip_clear_error();
  }
}

static Image from_oracle(OImage h) {
  Image im = new_image(h.width, h.height, (UphipPixelFormat)h.format, CP(Pixel, h.background),
                       h.abs_black_threshold);
  for (int y = 0; y < h.height; y++)
    memcpy(im.frame->data + (int64_t)y * im.frame->linesize, h.data + (int64_t)y * h.linesize,
           (size_t)o_min_linesize(h.width, h.format));
  return im;
}

/* ensure_cpu, then the visible pixels against the oracle's */
static void compare(const char *op, OImage h, Image *im) {
  g_checks++;
  if (getenv("ADAPTER_TRACE")) fprintf(stderr, "check %s [%s]\n", op, fmt_name(h.format));
  api_error(op);
  backend_hip_ensure_cpu(im);
  api_error("ensure_cpu");
  if (getenv("ADAPTER_TRACE")) fprintf(stderr, "  downloaded\n");
  const AVFrame *f = im->frame;
  if (f->width != h.width || f->height != h.height || (int)f->format != h.format) {
    fprintf(stderr, "MISMATCH %s [%s]: geometry %dx%d vs %dx%d\n", op, fmt_name(h.format),
            f->width, f->height, h.width, h.height);
    g_failures++;
    return;
  }
  const bool mono = h.format == UPHIP_FMT_MONOWHITE || h.format == UPHIP_FMT_MONOBLACK;
  for (int y = 0; y < h.height; y++) {
    const uint8_t *a = h.data + (int64_t)y * h.linesize, *b = f->data + (int64_t)y * f->linesize;
    for (int x = 0; x < (mono ? h.width : (int)o_min_linesize(h.width, h.format)); x++) {
      const bool diff = mono ? (((a[x >> 3] ^ b[x >> 3]) >> (7 - (x & 7))) & 1) : a[x] != b[x];
      if (diff) {
        fprintf(stderr, "MISMATCH %s [%s]: %s %d of row %d\n", op, fmt_name(h.format),
                mono ? "pixel" : "byte", x, y);
        g_failures++;
        return;
      }
    }
  }
}

static void check_int(const char *op, int fmt, long long a, long long b, const char *what) {
  g_checks++;
  if (a != b) {
    fprintf(stderr, "MISMATCH %s [%s]: %s: %lld (oracle) vs %lld (adapter)\n", op, fmt_name(fmt),
            what, a, b);
    g_failures++;
  }
}

static UphipRectangle urect(int x0, int y0, int x1, int y1) {
  return (UphipRectangle){{{x0, y0}, {x1, y1}}};
}
static Rectangle rect(int x0, int y0, int x1, int y1) {
  return (Rectangle){{{x0, y0}, {x1, y1}}};
}

#define W0 600
#define H0 850

/* a host-side edit of both copies: a scribbled rectangle, then mark_cpu_dirty */
static void host_edit(OImage h, Image *im) {
  backend_hip_ensure_cpu(im);
  const int64_t rb = o_min_linesize(h.width, h.format);
  for (int y = 200; y < 260; y++) {
    memset(h.data + (int64_t)y * h.linesize + rb / 4, 0x00, (size_t)(rb / 8));
    memset(im->frame->data + (int64_t)y * im->frame->linesize + rb / 4, 0x00, (size_t)(rb / 8));
  }
  backend_hip_mark_cpu_dirty(im);
}

static void run_format(int fmt, const UphipOptions *o) {
  const UphipPixel ucolor = fmt == UPHIP_FMT_RGB24 ? (UphipPixel){200, 30, 40} : (UphipPixel){0, 0, 0};
  const Pixel color = CP(Pixel, ucolor);
  OImage h = host_page(fmt, W0, H0, 3); /* page 3: the dark band */
  Image im = from_oracle(h);

  o_wipe_rectangle(h, urect(10, 20, 200, 150), ucolor); /* 1 */
  wipe_rectangle_hip(im, rect(10, 20, 200, 150), color);
  compare("wipe_rectangle", h, &im);
  host_edit(h, &im);

  { /* 2 copy_rectangle, 3 center_image: a second frame, filled on the host */
    OImage ht = o_create_image((UphipRectangleSize){W0 - 100, H0 - 50}, fmt, true, h.background, 170);
    Image t = from_oracle(ht);
    o_copy_rectangle(h, ht, urect(30, 40, 400, 500), (UphipPoint){-5, 17});
    copy_rectangle_hip(im, t, rect(30, 40, 400, 500), (Point){-5, 17});
    compare("copy_rectangle", ht, &t);
    o_center_image(h, ht, (UphipPoint){0, 0}, (UphipRectangleSize){W0 - 100, H0 - 50});
    center_image_hip(im, t, (Point){0, 0}, (RectangleSize){W0 - 100, H0 - 50});
    compare("center_image", ht, &t);
    o_free_image(&ht);
    free_img(&t);
  }
  /* 4 stretch, 5 resize, 6 flip_rotate_90, 7 mirror, 8 shift: replaced frames */
  o_stretch_and_replace(&h, (UphipRectangleSize){W0 * 3 / 4, H0 * 5 / 4}, UPHIP_INTERP_CUBIC);
  stretch_and_replace_hip(&im, (RectangleSize){W0 * 3 / 4, H0 * 5 / 4}, INTERP_CUBIC);
  compare("stretch_and_replace", h, &im);
  o_resize_and_replace(&h, (UphipRectangleSize){W0 + 37, H0 - 20}, UPHIP_INTERP_LINEAR);
  resize_and_replace_hip(&im, (RectangleSize){W0 + 37, H0 - 20}, INTERP_LINEAR);
  compare("resize_and_replace", h, &im);
  o_flip_rotate_90(&h, 1);
  flip_rotate_90_hip(&im, 1);
  compare("flip_rotate_90", h, &im);
  host_edit(h, &im);
  o_mirror(h, (UphipDirection){true, true});
  mirror_hip(im, (Direction){true, true});
  compare("mirror", h, &im);
  o_shift_image(&h, (UphipDelta){13, -7});
  shift_image_hip(&im, (Delta){13, -7});
  compare("shift_image", h, &im);
  o_free_image(&h);
  free_img(&im);

  h = host_page(fmt, W0, H0, 3);
  im = from_oracle(h);
  { /* 9 apply_masks, 10 apply_wipes, 11 apply_border */
    const UphipRectangle um[2] = {urect(100, 100, 500, 700), urect(-20, 650, 300, 900)};
    Rectangle m[2];
    memcpy(m, um, sizeof m);
    o_apply_masks(h, um, 2, ucolor);
    apply_masks_hip(im, m, 2, color);
    compare("apply_masks", h, &im);
    UphipWipes uw;
    memset(&uw, 0, sizeof uw);
    uw.count = 2;
    uw.areas[0] = urect(0, 0, 50, 60);
    uw.areas[1] = urect(580, 800, 700, 900);
    o_apply_wipes(h, &uw, ucolor);
    apply_wipes_hip(im, CP(Wipes, uw), color);
    compare("apply_wipes", h, &im);
    o_apply_border(h, (UphipBorder){5, 6, 7, 8}, ucolor);
    apply_border_hip(im, (Border){5, 6, 7, 8}, color);
    compare("apply_border", h, &im);
  }
  { /* 12 detect_masks, 13 align_mask, 14 detect_border */
    UphipMaskDetectionParameters mp = o->mask_detection_parameters;
    const UphipPoint upts[2] = {{W0 / 2, H0 / 2}, {W0 / 4, H0 / 3}};
    Point pts[2];
    memcpy(pts, upts, sizeof pts);
    UphipRectangle mh[2];
    Rectangle md[2];
    const size_t nh = o_detect_masks(h, &mp, upts, 2, mh);
    const size_t nd = detect_masks_hip(im, CP(MaskDetectionParameters, mp), pts, 2, md);
    api_error("detect_masks");
    check_int("detect_masks", fmt, (long long)nh, (long long)nd, "count");
    for (size_t i = 0; i < nh && i < 2; i++) {
      check_int("detect_masks", fmt, mh[i].vertex[0].x, md[i].vertex[0].x, "x0");
      check_int("detect_masks", fmt, mh[i].vertex[1].y, md[i].vertex[1].y, "y1");
    }
    const UphipMaskAlignmentParameters ap = {{true, true, false, false}, {10, 12}};
    o_align_mask(h, mh[0], urect(0, 0, W0 - 1, H0 - 1), ap);
    align_mask_hip(im, CP(Rectangle, mh[0]), rect(0, 0, W0 - 1, H0 - 1),
                   CP(MaskAlignmentParameters, ap));
    compare("align_mask", h, &im);
    UphipBorderScanParameters bp = o->border_scan_parameters;
    bp.scan_direction = (UphipDirection){true, true};
    const UphipBorder bh = o_detect_border(h, bp, urect(0, 0, W0 - 1, H0 - 1));
    const Border bd = detect_border_hip(im, CP(BorderScanParameters, bp), rect(0, 0, W0 - 1, H0 - 1));
    api_error("detect_border");
    check_int("detect_border", fmt, bh.left, bd.left, "left");
    check_int("detect_border", fmt, bh.top, bd.top, "top");
    check_int("detect_border", fmt, bh.right, bd.right, "right");
    check_int("detect_border", fmt, bh.bottom, bd.bottom, "bottom");
  }
  o_free_image(&h);
  free_img(&im);

  h = host_page(fmt, W0, H0, 3);
  im = from_oracle(h);
  { /* 15 blackfilter (exclusions through the reference's pointer), 16-18 */
    UphipBlackfilterParameters ub = o->blackfilter_parameters;
    ub.exclusions_count = 1;
    ub.exclusions[0] = urect(0, 0, 120, 120);
    BlackfilterParameters rb;
    memcpy(&rb, &ub, offsetof(BlackfilterParameters, exclusions_count));
    Rectangle excl[1] = {rect(0, 0, 120, 120)};
    rb.exclusions_count = 1;
    rb.exclusions = excl;
    o_blackfilter(h, &ub);
    blackfilter_hip(im, rb);
    compare("blackfilter", h, &im);
    host_edit(h, &im);
    o_noisefilter(h, o->noisefilter_intensity, o->abs_white_threshold);
    noisefilter_hip(im, o->noisefilter_intensity, o->abs_white_threshold);
    compare("noisefilter", h, &im);
    o_blurfilter(h, o->blurfilter_parameters, o->abs_white_threshold);
    blurfilter_hip(im, CP(BlurfilterParameters, o->blurfilter_parameters), o->abs_white_threshold);
    compare("blurfilter", h, &im);
    o_grayfilter(h, o->grayfilter_parameters);
    grayfilter_hip(im, CP(GrayfilterParameters, o->grayfilter_parameters));
    compare("grayfilter", h, &im);
  }
  o_free_image(&h);
  free_img(&im);

  h = host_page(fmt, W0, H0, 5);
  im = from_oracle(h);
  { /* 19 detect_rotation, 20 deskew */
    const UphipRectangle um = urect(60, 80, W0 - 61, H0 - 81);
    UphipDeskewParameters dp = o->deskew_parameters;
    const float rh = o_detect_rotation(h, um, &dp);
    const float rd = detect_rotation_hip(im, CP(Rectangle, um), CP(DeskewParameters, dp));
    api_error("detect_rotation");
    uint32_t bh, bd;
    memcpy(&bh, &rh, 4);
    memcpy(&bd, &rd, 4);
    check_int("detect_rotation", fmt, bh, bd, "float bits");
    const float rad = rh != 0.0f ? rh : 0.0123f;
    o_deskew(h, um, rad, UPHIP_INTERP_CUBIC);
    deskew_hip(im, CP(Rectangle, um), rad, INTERP_CUBIC);
    compare("deskew", h, &im);
  }
  if (fmt == UPHIP_FMT_GRAY8 || fmt == UPHIP_FMT_RGB24) {
    /* the GPU output branch (nvimgcodec_encode_to_file's peer): the file
     * equals the oracle's encode of the same (compared) pixels */
    char path[128];
    snprintf(path, sizeof path, "/tmp/adapter_ops_%d_%d.jpg", (int)getpid(), fmt);
    const bool ok = backend_hip_encode_to_file(&im, 85, path);
    api_error("encode_to_file");
    const int64_t cap = (int64_t)h.width * h.height * 8 + 65536;
    uint8_t *exp = malloc((size_t)cap), *got = malloc((size_t)cap);
    const int64_t ne = o_jpeg_encode(h.data, h.linesize, h.width, h.height, fmt, 85, 0, exp, cap);
    FILE *f = ok ? fopen(path, "rb") : NULL;
    const int64_t ng = f ? (int64_t)fread(got, 1, (size_t)cap, f) : -1;
    if (f) fclose(f);
    remove(path);
    check_int("encode_to_file", fmt, ne, ng, "file size");
    check_int("encode_to_file", fmt, 0, ng == ne ? memcmp(exp, got, (size_t)ne) != 0 : 1, "bytes");
    free(exp);
    free(got);
  }
  o_free_image(&h);
  free_img(&im);
}

int main(void) {
  const UphipInitStatus st = uphip_try_init();
  if (st != UPHIP_INIT_OK) {
    fprintf(stderr, "adapter_ops: no HIP device (%s)\n", uphip_init_status_string(st));
    return 2;
  }
  UphipOptions o;
  uphip_options_init(&o);
  for (int fmt = UPHIP_FMT_GRAY8; fmt <= UPHIP_FMT_MONOBLACK; fmt++) run_format(fmt, &o);
  printf("adapter_ops: 20 ops on reference types x 5 formats, %d checks, %d mismatches\n",
         g_checks, g_failures);
  return g_failures ? 1 : 0;
}
