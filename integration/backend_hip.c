/* backend_hip.c — imageprocess/backend_hip.c for unpaper-gpu: the 20
 * ImageBackend ops (imageprocess/backend.h:22-56) on the reference's own
 * `Image` and value types, forwarded to libunpaper_hip.so.
 *
 * The reference's types and ours are layout-identical (checked below with
 * sizeof and offsetof at compile time), so parameters are copied bit for bit,
 * not converted field by field; the one exception is BlackfilterParameters, whose exclusions are
 * a caller-owned pointer in the reference (filters.h:27-28) and an inline
 * array at the C ABI.
 *
 * Residency follows image_cuda.c:109-305: each frame carries a HipState
 * (hip_frame.h) with a device copy that is uploaded when the host bytes are
 * newer and marked newer than the host after every writing op;
 * backend_hip_ensure_cpu() downloads it for the CPU stages and the encoder.
 *
 * This file compiles against the reference headers as they are
 * (`gcc -I<reference> -I<repo>/include -I<repo>/integration -c`); the
 * AVFrame-touching hooks and the vtable instance are in backend_hip_av.c.
 */
#include "backend_hip.h"

#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "unpaper_hip.h"

#define SAME_LAYOUT(R, U) _Static_assert(sizeof(R) == sizeof(U), #R " size")
#define SAME_FIELD(R, U, f) \
  _Static_assert(offsetof(R, f) == offsetof(U, f), #R "." #f " offset")

SAME_LAYOUT(Point, UphipPoint);
SAME_FIELD(Point, UphipPoint, y);
SAME_LAYOUT(Delta, UphipDelta);
SAME_FIELD(Delta, UphipDelta, vertical);
SAME_LAYOUT(Direction, UphipDirection);
SAME_FIELD(Direction, UphipDirection, vertical);
SAME_LAYOUT(Edges, UphipEdges);
SAME_FIELD(Edges, UphipEdges, bottom);
SAME_LAYOUT(Pixel, UphipPixel);
SAME_FIELD(Pixel, UphipPixel, b);
SAME_LAYOUT(Rectangle, UphipRectangle);
SAME_LAYOUT(RectangleSize, UphipRectangleSize);
SAME_FIELD(RectangleSize, UphipRectangleSize, height);
SAME_LAYOUT(Border, UphipBorder);
SAME_FIELD(Border, UphipBorder, bottom);
SAME_LAYOUT(Wipes, UphipWipes);
SAME_FIELD(Wipes, UphipWipes, areas);
SAME_LAYOUT(Interpolation, UphipInterpolation);
SAME_LAYOUT(RotationDirection, UphipRotationDirection);
SAME_LAYOUT(BlurfilterParameters, UphipBlurfilterParameters);
SAME_FIELD(BlurfilterParameters, UphipBlurfilterParameters, scan_step);
SAME_FIELD(BlurfilterParameters, UphipBlurfilterParameters, intensity);
SAME_LAYOUT(GrayfilterParameters, UphipGrayfilterParameters);
SAME_FIELD(GrayfilterParameters, UphipGrayfilterParameters, abs_threshold);
SAME_LAYOUT(MaskDetectionParameters, UphipMaskDetectionParameters);
SAME_FIELD(MaskDetectionParameters, UphipMaskDetectionParameters, scan_depth);
SAME_FIELD(MaskDetectionParameters, UphipMaskDetectionParameters, scan_direction);
SAME_FIELD(MaskDetectionParameters, UphipMaskDetectionParameters, scan_threshold);
SAME_FIELD(MaskDetectionParameters, UphipMaskDetectionParameters, minimum_width);
SAME_FIELD(MaskDetectionParameters, UphipMaskDetectionParameters, maximum_height);
SAME_LAYOUT(MaskAlignmentParameters, UphipMaskAlignmentParameters);
SAME_FIELD(MaskAlignmentParameters, UphipMaskAlignmentParameters, margin);
SAME_LAYOUT(BorderScanParameters, UphipBorderScanParameters);
SAME_FIELD(BorderScanParameters, UphipBorderScanParameters, scan_threshold);
SAME_FIELD(BorderScanParameters, UphipBorderScanParameters, scan_direction);
SAME_LAYOUT(DeskewParameters, UphipDeskewParameters);
SAME_FIELD(DeskewParameters, UphipDeskewParameters, deskewScanSize);
SAME_FIELD(DeskewParameters, UphipDeskewParameters, deskewScanDepth);
SAME_FIELD(DeskewParameters, UphipDeskewParameters, scan_edges);
/* everything of BlackfilterParameters before the exclusions */
SAME_FIELD(BlackfilterParameters, UphipBlackfilterParameters, scan_depth);
SAME_FIELD(BlackfilterParameters, UphipBlackfilterParameters, scan_direction);
SAME_FIELD(BlackfilterParameters, UphipBlackfilterParameters, abs_threshold);
SAME_FIELD(BlackfilterParameters, UphipBlackfilterParameters, intensity);
SAME_FIELD(BlackfilterParameters, UphipBlackfilterParameters, exclusions_count);
_Static_assert(MAX_MASKS == UPHIP_MAX_MASKS, "MAX_MASKS");
_Static_assert(INTERP_NN == (int)UPHIP_INTERP_NN && INTERP_LINEAR == (int)UPHIP_INTERP_LINEAR &&
                   INTERP_CUBIC == (int)UPHIP_INTERP_CUBIC,
               "Interpolation values");

/* layout-identical value types: copied bit for bit (memcpy, so no type
 * punning through pointers); arrays are passed on as they are */
#define AS(T, v)                    \
  ({                                \
    T as_;                          \
    memcpy(&as_, &(v), sizeof as_); \
    as_;                            \
  })
#define ASP(T, p) ((const T *)(p))

/* ------------------------------------------------------------------------- */
/* residency                                                                 */
/* ------------------------------------------------------------------------- */

/* The device copy of `image`, uploaded when the host bytes are newer
 * (image_ensure_cuda, image_cuda.c:135-206).  Background and threshold travel
 * with the Image value, so they are refreshed on every call. */
static UphipImage dev(Image image) {
  HipState *st = hip_state(image.frame);
  if (!st->img.frame) {
    const HipFrameView v = hip_frame_view(image.frame);
    st->img = uphip_create_image((UphipRectangleSize){v.width, v.height}, v.format, false,
                                 AS(UphipPixel, image.background), image.abs_black_threshold);
    st->host_newer = true;
  }
  if (st->host_newer) {
    const HipFrameView v = hip_frame_view(image.frame);
    uphip_image_upload(st->img, v.data, v.linesize);
    st->host_newer = false;
  }
  UphipImage d = st->img;
  d.background = AS(UphipPixel, image.background);
  d.abs_black_threshold = image.abs_black_threshold;
  return d;
}

/* after a writing op (image_mark_cuda_dirty, image_cuda.c:122-133) */
static void wrote(Image image) { hip_state(image.frame)->device_newer = true; }

/* after an op on *pImage that may change its geometry.  The library either
 * re-stores the same handle (adopt_storage in ops.hip) or hands back a new one
 * (uphip_replace_image); either way `d` now owns the device pixels.  Same size:
 * the frame keeps them; new size: a new frame of that size adopts them. */
static void replaced(Image *pImage, UphipImage d) {
  HipState *st = hip_state(pImage->frame);
  const HipFrameView v = hip_frame_view(pImage->frame);
  const UphipRectangleSize s = uphip_size_of_image(d);
  if (s.width == v.width && s.height == v.height) {
    st->img.frame = d.frame;
    st->device_newer = true;
    return;
  }
  st->img.frame = NULL; /* owned by `d` from here on */
  hip_adopt(pImage, d);
}

void backend_hip_ensure_cpu(Image *image) {
  if (!image || !image->frame) return;
  HipState *st = hip_state(image->frame);
  if (!st->img.frame || !st->device_newer) return;
  const HipFrameView v = hip_frame_view(image->frame);
  uphip_image_download(st->img, v.data, v.linesize);
  st->device_newer = false;
}

void backend_hip_mark_cpu_dirty(Image *image) {
  if (!image || !image->frame) return;
  HipState *st = hip_state(image->frame);
  st->host_newer = true;
  st->device_newer = false;
}

void backend_hip_mark_gpu_dirty(Image *image) {
  if (!image || !image->frame) return;
  HipState *st = hip_state(image->frame);
  st->device_newer = true;
  st->host_newer = false;
}

void backend_hip_release(HipState *st) {
  if (st && st->img.frame) uphip_free_image(&st->img);
}

/* ------------------------------------------------------------------------- */
/* the 20 ops, backend.h:22-56                                               */
/* ------------------------------------------------------------------------- */

void wipe_rectangle_hip(Image image, Rectangle input_area, Pixel color) {
  uphip_wipe_rectangle(dev(image), AS(UphipRectangle, input_area), AS(UphipPixel, color));
  wrote(image);
}

void copy_rectangle_hip(Image source, Image target, Rectangle source_area, Point target_coords) {
  uphip_copy_rectangle(dev(source), dev(target), AS(UphipRectangle, source_area),
                       AS(UphipPoint, target_coords));
  wrote(target);
}

void center_image_hip(Image source, Image target, Point target_origin, RectangleSize target_size) {
  uphip_center_image(dev(source), dev(target), AS(UphipPoint, target_origin),
                     AS(UphipRectangleSize, target_size));
  wrote(target);
}

void stretch_and_replace_hip(Image *pImage, RectangleSize size, Interpolation interpolate_type) {
  UphipImage d = dev(*pImage);
  uphip_stretch_and_replace(&d, AS(UphipRectangleSize, size), (UphipInterpolation)interpolate_type);
  replaced(pImage, d);
}

void resize_and_replace_hip(Image *pImage, RectangleSize size, Interpolation interpolate_type) {
  UphipImage d = dev(*pImage);
  uphip_resize_and_replace(&d, AS(UphipRectangleSize, size), (UphipInterpolation)interpolate_type);
  replaced(pImage, d);
}

void flip_rotate_90_hip(Image *pImage, RotationDirection direction) {
  UphipImage d = dev(*pImage);
  uphip_flip_rotate_90(&d, (UphipRotationDirection)direction);
  replaced(pImage, d);
}

void mirror_hip(Image image, Direction direction) {
  uphip_mirror(dev(image), AS(UphipDirection, direction));
  wrote(image);
}

void shift_image_hip(Image *pImage, Delta d) {
  UphipImage im = dev(*pImage);
  uphip_shift_image(&im, AS(UphipDelta, d));
  replaced(pImage, im);
}

void apply_masks_hip(Image image, const Rectangle masks[], size_t masks_count, Pixel color) {
  uphip_apply_masks(dev(image), ASP(UphipRectangle, masks), masks_count, AS(UphipPixel, color));
  wrote(image);
}

void apply_wipes_hip(Image image, Wipes wipes, Pixel color) {
  uphip_apply_wipes(dev(image), AS(UphipWipes, wipes), AS(UphipPixel, color));
  wrote(image);
}

void apply_border_hip(Image image, const Border border, Pixel color) {
  uphip_apply_border(dev(image), AS(UphipBorder, border), AS(UphipPixel, color));
  wrote(image);
}

size_t detect_masks_hip(Image image, MaskDetectionParameters params, const Point points[],
                        size_t points_count, Rectangle masks[]) {
  return uphip_detect_masks(dev(image), AS(UphipMaskDetectionParameters, params),
                            ASP(UphipPoint, points), points_count, (UphipRectangle *)masks);
}

void align_mask_hip(Image image, const Rectangle inside_area, const Rectangle outside,
                    MaskAlignmentParameters params) {
  uphip_align_mask(dev(image), AS(UphipRectangle, inside_area), AS(UphipRectangle, outside),
                   AS(UphipMaskAlignmentParameters, params));
  wrote(image);
}

Border detect_border_hip(Image image, BorderScanParameters params, const Rectangle outside_mask) {
  const UphipBorder b = uphip_detect_border(dev(image), AS(UphipBorderScanParameters, params),
                                            AS(UphipRectangle, outside_mask));
  return AS(Border, b);
}

void blackfilter_hip(Image image, BlackfilterParameters params) {
  UphipBlackfilterParameters q;
  memset(&q, 0, sizeof q);
  memcpy(&q, &params, offsetof(BlackfilterParameters, exclusions_count));
  /* the reference takes any count through its pointer; the C ABI holds
   * MAX_MASKS inline, the most the option parser accepts
   * (cli_options.c:707, options.h:124) */
  q.exclusions_count = params.exclusions_count < UPHIP_MAX_MASKS ? params.exclusions_count
                                                                 : UPHIP_MAX_MASKS;
  if (q.exclusions_count && params.exclusions)
    memcpy(q.exclusions, params.exclusions, q.exclusions_count * sizeof(Rectangle));
  else
    q.exclusions_count = 0;
  uphip_blackfilter(dev(image), q);
  wrote(image);
}

void blurfilter_hip(Image image, BlurfilterParameters params, uint8_t abs_white_threshold) {
  uphip_blurfilter(dev(image), AS(UphipBlurfilterParameters, params), abs_white_threshold);
  wrote(image);
}

void noisefilter_hip(Image image, uint64_t intensity, uint8_t min_white_level) {
  uphip_noisefilter(dev(image), intensity, min_white_level);
  wrote(image);
}

void grayfilter_hip(Image image, GrayfilterParameters params) {
  uphip_grayfilter(dev(image), AS(UphipGrayfilterParameters, params));
  wrote(image);
}

float detect_rotation_hip(Image image, Rectangle mask, const DeskewParameters params) {
  return uphip_detect_rotation(dev(image), AS(UphipRectangle, mask),
                               AS(UphipDeskewParameters, params));
}

void deskew_hip(Image source, Rectangle mask, float radians, Interpolation interpolate_type) {
  uphip_deskew(dev(source), AS(UphipRectangle, mask), radians,
               (UphipInterpolation)interpolate_type);
  wrote(source);
}

/* The GPU output branch (sheet_stages.c:554-581 -> encode_queue_submit_gpu,
 * lib/encode_queue.c:860-990): the sheet's device copy encoded as a JPEG
 * file, the peer of nvimgcodec_encode_to_file (nvimgcodec.c:1164-1200).
 * quality 0 = 85 (lib/options.h:42).  GRAY8 sheets give one component,
 * RGB24 sheets YCbCr 4:4:4. */
bool backend_hip_encode_to_file(Image *image, int quality, const char *filename) {
  const UphipImage d = dev(*image);
  const void *src = uphip_image_device_ptr(d);
  const int64_t pitch = uphip_image_device_pitch(d);
  const UphipRectangleSize sz = uphip_size_of_image(d);
  const UphipPixelFormat fmt = uphip_image_format(d);
  if (!src || (fmt != UPHIP_FMT_GRAY8 && fmt != UPHIP_FMT_RGB24)) return false;
  const int64_t n = uphip_jpeg_encode(src, pitch, sz.width, sz.height, fmt, quality,
                                      UPHIP_JPEG_444, NULL, 0);
  if (n <= 0) return false;
  uint8_t *buf = malloc((size_t)n);
  if (!buf) return false;
  bool ok = uphip_jpeg_encode(src, pitch, sz.width, sz.height, fmt, quality, UPHIP_JPEG_444,
                              buf, n) == n;
  FILE *f = ok ? fopen(filename, "wb") : NULL;
  ok = f && fwrite(buf, 1, (size_t)n, f) == (size_t)n;
  if (f && fclose(f) != 0) ok = false;
  free(buf);
  return ok;
}

