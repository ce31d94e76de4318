// ops.hip — the ImageBackend ops (imageprocess/backend.h:22-56) over device
// frames, one batch-of-one launch sequence per call.  Argument meaning, clipping
// and error behaviour follow the CPU implementations cited per function; ops
// that return values synchronise the current stream.
#include <cmath>
#include <cstdio>
#include <vector>

#include "filters.h"
#include "mono_proxy.h"
#include "runtime.h"
#include "scan.h"

namespace uph {

void launch_fill_thr(const PlaneRef& dst, const FillArgs* args, int count, int rows_hint,
                     uint8_t thr, hipStream_t st);
void launch_copy_thr(const PlaneRef& src, const PlaneRef& dst, const CopyArgs* args, int count,
                     int rows_hint, uint8_t thr, hipStream_t st);
void launch_apply_masks_thr(const PlaneRef& dst, const MaskArgs* args, int count, uint8_t thr,
                            hipStream_t st);
void launch_mirror_oop(const PlaneRef& src, const PlaneRef& dst, bool h, bool v, uint8_t thr,
                       int count, hipStream_t st);
void launch_rotate90_thr(const PlaneRef& src, const PlaneRef& dst, int direction, uint8_t thr,
                         int count, hipStream_t st);
void launch_stretch_thr(const PlaneRef& src, const PlaneRef& dst, int interp, uint8_t thr,
                        int count, hipStream_t st);

static bool ok_image(const UphipImage& im, const char* op) {
  if (!im.frame) return fail("%s: image has no frame", op);
  if (!runtime_ready()) return fail("%s: no HIP device", op);
  hipSetDevice(im.frame->device);
  return true;
}

static PlaneRef ref_of(const UphipFrame* f) { return fixed_ref(frame_planes(f), 0); }

static void fill_frame(UphipFrame* f, Rect clipped, Px c, uint8_t thr, hipStream_t st) {
  if (clipped.x1 < clipped.x0 || clipped.y1 < clipped.y0) return;
  FillArgs a{clipped, {c.r, c.g, c.b}, 1};
  FillArgs* d = stage_args(&a, 1, st);
  if (!d) return;
  launch_fill_thr(ref_of(f), d, 1, clipped.y1 - clipped.y0 + 1, thr, st);
  arg_fence(st);
}

static void copy_frames(const UphipFrame* src, UphipFrame* dst, Rect clipped, int32_t tx,
                        int32_t ty, uint8_t thr, hipStream_t st) {
  if (clipped.x1 < clipped.x0 || clipped.y1 < clipped.y0) return;
  CopyArgs a{clipped, tx, ty, 1};
  CopyArgs* d = stage_args(&a, 1, st);
  if (!d) return;
  launch_copy_thr(ref_of(src), ref_of(dst), d, 1, clipped.y1 - clipped.y0 + 1, thr, st);
  arg_fence(st);
}

// Replace the frame's storage by `n`'s (the UphipFrame object stays, so every
// UphipImage copy that points at it sees the new pixels).
static void adopt_storage(UphipFrame* f, UphipFrame* n) {
  hipStreamSynchronize(current_stream());
  hipFree(f->data);
  *f = *n;
  delete n;
}

}  // namespace uph

using namespace uph;

extern "C" {

// ---------------------------------------------------------------------------
// image.c peers
// ---------------------------------------------------------------------------
UphipImage uphip_create_image(UphipRectangleSize size, UphipPixelFormat format, bool fill,
                              UphipPixel background, uint8_t abs_black_threshold) {
  UphipImage im{nullptr, background, abs_black_threshold};
  im.frame = frame_alloc(size.width, size.height, format);
  if (im.frame && fill)
    fill_frame(im.frame, Rect{0, 0, size.width - 1, size.height - 1},
               Px{background.r, background.g, background.b}, abs_black_threshold,
               current_stream());
  return im;
}

void uphip_free_image(UphipImage* image) {
  if (!image) return;
  frame_free(image->frame);
  image->frame = nullptr;
}

void uphip_replace_image(UphipImage* image, UphipImage* new_image) {
  uphip_free_image(image);
  *image = *new_image;
  new_image->frame = nullptr;
}

UphipImage uphip_create_compatible_image(UphipImage source, UphipRectangleSize size, bool fill) {
  return uphip_create_image(size, (UphipPixelFormat)source.frame->format, fill, source.background,
                            source.abs_black_threshold);
}

UphipRectangleSize uphip_size_of_image(UphipImage image) {
  UphipRectangleSize s{0, 0};
  if (image.frame) s = UphipRectangleSize{image.frame->width, image.frame->height};
  return s;
}

UphipPixelFormat uphip_image_format(UphipImage image) {
  return image.frame ? (UphipPixelFormat)image.frame->format : UPHIP_FMT_NONE;
}

int uphip_image_upload(UphipImage image, const void* host, int64_t linesize) {
  if (!ok_image(image, "upload")) return -1;
  UphipFrame* f = image.frame;
  const int64_t rb = row_bytes(f->width, f->format);
  if (linesize < rb) return fail("upload: linesize %lld < row bytes %lld", (long long)linesize,
                                 (long long)rb), -1;
  hipStream_t st = current_stream();
  if (!UPH_HIP(hipMemcpy2DAsync(f->data, f->pitch, host, linesize, rb, f->height,
                                hipMemcpyHostToDevice, st)))
    return -1;
  return UPH_HIP(hipStreamSynchronize(st)) ? 0 : -1;
}

int uphip_image_download(UphipImage image, void* host, int64_t linesize) {
  if (!ok_image(image, "download")) return -1;
  UphipFrame* f = image.frame;
  const int64_t rb = row_bytes(f->width, f->format);
  if (linesize < rb) return fail("download: linesize too small"), -1;
  hipStream_t st = current_stream();
  if (!UPH_HIP(hipMemcpy2DAsync(host, linesize, f->data, f->pitch, rb, f->height,
                                hipMemcpyDeviceToHost, st)))
    return -1;
  return UPH_HIP(hipStreamSynchronize(st)) ? 0 : -1;
}

void* uphip_image_device_ptr(UphipImage image) { return image.frame ? image.frame->data : nullptr; }
int64_t uphip_image_device_pitch(UphipImage image) { return image.frame ? image.frame->pitch : 0; }

// ---------------------------------------------------------------------------
// blit.c peers
// ---------------------------------------------------------------------------
void uphip_wipe_rectangle(UphipImage image, UphipRectangle input_area, UphipPixel color) {
  // wipe_rectangle_cpu, blit.c:20-24
  if (!ok_image(image, "wipe_rectangle")) return;
  UphipFrame* f = image.frame;
  fill_frame(f, clip(to_rect(input_area), f->width, f->height), Px{color.r, color.g, color.b},
             image.abs_black_threshold, current_stream());
}

void uphip_copy_rectangle(UphipImage source, UphipImage target, UphipRectangle source_area,
                          UphipPoint target_coords) {
  // copy_rectangle_cpu, blit.c:30-80
  if (!ok_image(source, "copy_rectangle") || !ok_image(target, "copy_rectangle")) return;
  if (source.frame->device != target.frame->device)
    return (void)fail("copy_rectangle: frames on different devices");
  Rect a = clip(to_rect(source_area), source.frame->width, source.frame->height);
  copy_frames(source.frame, target.frame, a, target_coords.x, target_coords.y,
              target.abs_black_threshold, current_stream());
}

void uphip_center_image(UphipImage source, UphipImage target, UphipPoint to,
                        UphipRectangleSize ts) {
  // center_image_cpu, blit.c:175-202
  if (!ok_image(source, "center_image") || !ok_image(target, "center_image")) return;
  UphipPoint so{0, 0};
  UphipRectangleSize ss{source.frame->width, source.frame->height};
  if (ss.width < ts.width || ss.height < ts.height)
    uphip_wipe_rectangle(target, from_rect(rect_from_size(to.x, to.y, ts.width, ts.height)),
                         target.background);
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
  uphip_copy_rectangle(source, target, from_rect(rect_from_size(so.x, so.y, ss.width, ss.height)),
                       to);
}

static int compare_sizes(UphipRectangleSize a, UphipRectangleSize b) {
  // primitives.c:70-80
  if (a.height == b.height && a.width == b.width) return 0;
  return imin(a.height, a.width) < imin(b.height, b.width) ? -1 : 1;
}

void uphip_stretch_and_replace(UphipImage* pImage, UphipRectangleSize size,
                               UphipInterpolation interp) {
  // stretch_and_replace_cpu, blit.c:231-239
  if (!pImage || !ok_image(*pImage, "stretch_and_replace")) return;
  UphipFrame* f = pImage->frame;
  if (compare_sizes(UphipRectangleSize{f->width, f->height}, size) == 0) return;
  UphipFrame* n = frame_alloc(size.width, size.height, f->format);
  if (!n) return;
  launch_stretch_thr(ref_of(f), ref_of(n), interp, pImage->abs_black_threshold, 1,
                     current_stream());
  adopt_storage(f, n);
}

void uphip_resize_and_replace(UphipImage* pImage, UphipRectangleSize size,
                              UphipInterpolation interp) {
  // resize_and_replace_cpu, blit.c:246-282
  if (!pImage || !ok_image(*pImage, "resize_and_replace")) return;
  UphipRectangleSize is{pImage->frame->width, pImage->frame->height};
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
  uphip_stretch_and_replace(pImage, ss, interp);
  if (size.width == ss.width && size.height == ss.height) return;
  UphipImage resized = uphip_create_compatible_image(*pImage, size, true);
  if (!resized.frame) return;
  uphip_center_image(*pImage, resized, UphipPoint{0, 0}, size);
  uphip_replace_image(pImage, &resized);
}

void uphip_flip_rotate_90(UphipImage* pImage, UphipRotationDirection direction) {
  // flip_rotate_90_cpu, blit.c:289-310
  if (!pImage || !ok_image(*pImage, "flip_rotate_90")) return;
  UphipFrame* f = pImage->frame;
  UphipFrame* n = frame_alloc(f->height, f->width, f->format);
  if (!n) return;
  launch_rotate90_thr(ref_of(f), ref_of(n), direction, pImage->abs_black_threshold, 1,
                      current_stream());
  adopt_storage(f, n);
}

void uphip_mirror(UphipImage image, UphipDirection direction) {
  // mirror_cpu, blit.c:316-349 (every pixel is re-written via set_pixel)
  if (!ok_image(image, "mirror")) return;
  UphipFrame* f = image.frame;
  UphipFrame* n = frame_alloc(f->width, f->height, f->format);
  if (!n) return;
  launch_mirror_oop(ref_of(f), ref_of(n), direction.horizontal, direction.vertical,
                    image.abs_black_threshold, 1, current_stream());
  adopt_storage(f, n);
}

void uphip_shift_image(UphipImage* pImage, UphipDelta d) {
  // shift_image_cpu, blit.c:355-363
  if (!pImage || !ok_image(*pImage, "shift_image")) return;
  UphipImage n = uphip_create_compatible_image(*pImage, uphip_size_of_image(*pImage), true);
  if (!n.frame) return;
  uphip_copy_rectangle(*pImage, n,
                       from_rect(Rect{0, 0, pImage->frame->width - 1, pImage->frame->height - 1}),
                       UphipPoint{d.horizontal, d.vertical});
  uphip_replace_image(pImage, &n);
}

// ---------------------------------------------------------------------------
// masks.c peers
// ---------------------------------------------------------------------------
void uphip_apply_masks(UphipImage image, const UphipRectangle masks[], size_t masks_count,
                       UphipPixel color) {
  // apply_masks_cpu, masks.c:306-322
  if (masks_count <= 0) return;
  if (!ok_image(image, "apply_masks")) return;
  if (masks_count > UPHIP_MAX_MASKS) return (void)fail("apply_masks: too many masks");
  MaskArgs a;
  a.n = (int32_t)masks_count;
  a.color[0] = color.r;
  a.color[1] = color.g;
  a.color[2] = color.b;
  for (size_t i = 0; i < masks_count; i++) a.m[i] = to_rect(masks[i]);
  hipStream_t st = current_stream();
  MaskArgs* d = stage_args(&a, 1, st);
  if (!d) return;
  launch_apply_masks_thr(ref_of(image.frame), d, 1, image.abs_black_threshold, st);
  arg_fence(st);
}

void uphip_apply_wipes(UphipImage image, UphipWipes wipes, UphipPixel color) {
  // apply_wipes_cpu, masks.c:333-345: scan_rectangle over the rectangle AS
  // GIVEN (an inverted one covers nothing); set_pixel drops outside pixels.
  if (!ok_image(image, "apply_wipes")) return;
  UphipFrame* f = image.frame;
  for (size_t i = 0; i < wipes.count && i < UPHIP_MAX_MASKS; i++) {
    Rect r = to_rect(wipes.areas[i]);
    if (r.x0 > r.x1 || r.y0 > r.y1) continue;
    fill_frame(f, clip(r, f->width, f->height), Px{color.r, color.g, color.b},
               image.abs_black_threshold, current_stream());
  }
}

static UphipRectangle border_to_mask(int32_t W, int32_t H, UphipBorder b) {
  // masks.c:351-366
  return from_rect(Rect{b.left, b.top, W - b.right - 1, H - b.bottom - 1});
}

void uphip_apply_border(UphipImage image, const UphipBorder border, UphipPixel color) {
  // apply_border_cpu, masks.c:372-383
  if (border.left == 0 && border.top == 0 && border.right == 0 && border.bottom == 0) return;
  if (!ok_image(image, "apply_border")) return;
  UphipRectangle m = border_to_mask(image.frame->width, image.frame->height, border);
  uphip_apply_masks(image, &m, 1, color);
}

size_t uphip_detect_masks(UphipImage image0, UphipMaskDetectionParameters params,
                          const UphipPoint points[], size_t points_count,
                          UphipRectangle masks[]) {
  // detect_masks_cpu / detect_mask / detect_edge, masks.c:54-209
  if (!params.scan_direction.horizontal && !params.scan_direction.vertical) return 0;
  if (points_count == 0) return 0;
  if (!ok_image(image0, "detect_masks")) return 0;
  MonoProxy mp(image0, false, "detect_masks");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return 0;
  const UphipImage image = mp.image();
  UphipFrame* f = image.frame;
  const int32_t W = f->width, H = f->height;
  hipStream_t st = current_stream();
  // one axis-sum row per (point, direction); edges: 4 per point
  const size_t n = points_count;
  std::vector<AxisArgs> col_args, row_args;
  std::vector<EdgeArgs> edges(4 * n);
  const int32_t stride = imax(W, H);
  uint32_t* sums = (uint32_t*)scratch(0, sizeof(uint32_t) * stride * 2 * n);
  int32_t* res = (int32_t*)scratch(1, sizeof(int32_t) * 4 * n);
  if (!sums || !res) return 0;
  UPH_HIP(hipMemsetAsync(sums, 0, sizeof(uint32_t) * stride * 2 * n, st));
  for (size_t i = 0; i < n; i++) {
    const UphipPoint o = points[i];
    EdgeArgs* e = &edges[4 * i];
    for (int k = 0; k < 4; k++) e[k].active = 0;
    if (params.scan_direction.horizontal) {
      int32_t depth = params.scan_depth.horizontal == -1 ? H : params.scan_depth.horizontal;
      const int32_t size = params.scan_size.width;
      const int32_t c0 = o.y - depth / 2, c1 = c0 + depth - 1;
      Rect reg = clip(Rect{0, c0, W - 1, c1}, W, H);
      AxisArgs aa{reg, 0, (reg.y1 >= reg.y0) ? 1 : 0};
      // each point gets its own sums row (index 2i): launched one by one below
      col_args.push_back(aa);
      for (int k = 0; k < 2; k++) {
        EdgeArgs& ea = e[k];
        ea.active = 1;
        ea.sums_offset = 0;
        ea.extent = W;
        ea.cross_extent = H;
        ea.c0 = c0;
        ea.c1 = c1;
        ea.b0 = o.x - size / 2;
        ea.step = (k == 0 ? -1 : 1) * params.scan_step.horizontal;
        ea.size = size;
        ea.threshold = params.scan_threshold.horizontal;
      }
    } else {
      col_args.push_back(AxisArgs{Rect{0, 0, -1, -1}, 0, 0});
    }
    if (params.scan_direction.vertical) {
      int32_t depth = params.scan_depth.vertical == -1 ? W : params.scan_depth.vertical;
      const int32_t size = params.scan_size.height;
      const int32_t c0 = o.x - depth / 2, c1 = c0 + depth - 1;
      Rect reg = clip(Rect{c0, 0, c1, H - 1}, W, H);
      row_args.push_back(AxisArgs{reg, 0, (reg.x1 >= reg.x0) ? 1 : 0});
      for (int k = 2; k < 4; k++) {
        EdgeArgs& ea = e[k];
        ea.active = 1;
        ea.sums_offset = 0;
        ea.extent = H;
        ea.cross_extent = W;
        ea.c0 = c0;
        ea.c1 = c1;
        ea.b0 = o.y - size / 2;
        ea.step = (k == 2 ? -1 : 1) * params.scan_step.vertical;
        ea.size = size;
        ea.threshold = params.scan_threshold.vertical;
      }
    } else {
      row_args.push_back(AxisArgs{Rect{0, 0, -1, -1}, 0, 0});
    }
  }
  // reductions: sums row 2i = columns (horizontal), 2i+1 = rows (vertical)
  for (size_t i = 0; i < n; i++) {
    AxisArgs* ca = stage_args(&col_args[i], 1, st);
    AxisArgs* ra = stage_args(&row_args[i], 1, st);
    if (!ca || !ra) return 0;
    if (col_args[i].active)
      launch_axis_reduce(ref_of(f), ca, 0, M_GRAY_SUM, W, H, sums + (2 * i) * stride, 0, 1, st);
    if (row_args[i].active)
      launch_axis_reduce(ref_of(f), ra, 1, M_GRAY_SUM, W, H, sums + (2 * i + 1) * stride, 0, 1,
                         st);
    arg_fence(st);
  }
  for (size_t i = 0; i < n; i++) {
    EdgeArgs* e = &edges[4 * i];
    e[0].sums_offset = e[1].sums_offset = (int32_t)((2 * i) * stride);
    e[2].sums_offset = e[3].sums_offset = (int32_t)((2 * i + 1) * stride);
  }
  EdgeArgs* de = stage_args(edges.data(), edges.size(), st);
  if (!de) return 0;
  launch_edge_scan(de, (int)edges.size(), sums, 0, res, 1, st, imax(W, H));
  arg_fence(st);
  std::vector<int32_t> counts(4 * n);
  UPH_HIP(hipMemcpyAsync(counts.data(), res, sizeof(int32_t) * 4 * n, hipMemcpyDeviceToHost, st));
  if (!UPH_HIP(hipStreamSynchronize(st))) return 0;
  size_t valid = 0;
  for (size_t i = 0; i < n; i++) {
    // detect_mask, masks.c:107-171
    const UphipPoint o = points[i];
    Rect m;
    if (params.scan_direction.horizontal) {
      m.x0 = o.x - (params.scan_step.horizontal * counts[4 * i]) - params.scan_size.width / 2;
      m.x1 = o.x + (params.scan_step.horizontal * counts[4 * i + 1]) + params.scan_size.width / 2;
    } else {
      m.x0 = 0;
      m.x1 = W - 1;
    }
    if (params.scan_direction.vertical) {
      m.y0 = o.y - (params.scan_step.vertical * counts[4 * i + 2]) - params.scan_size.height / 2;
      m.y1 = o.y + (params.scan_step.vertical * counts[4 * i + 3]) + params.scan_size.height / 2;
    } else {
      m.y0 = 0;
      m.y1 = H - 1;
    }
    const int32_t mw = iabs(m.x0 - m.x1) + 1, mh = iabs(m.y0 - m.y1) + 1;
    if ((params.minimum_width != -1 && mw < params.minimum_width) ||
        (params.maximum_width != -1 && mw > params.maximum_width)) {
      m.x0 = o.x - params.maximum_width / 2;
      m.x1 = o.x + params.maximum_width / 2;
    }
    if ((params.minimum_height != -1 && mh < params.minimum_height) ||
        (params.maximum_height != -1 && mh > params.maximum_height)) {
      m.y0 = o.y - params.maximum_height / 2;
      m.y1 = o.y + params.maximum_height / 2;
    }
    masks[i] = from_rect(m);
    if (!(m.x0 == -1 && m.y0 == -1 && m.x1 == -1 && m.y1 == -1)) valid++;
  }
  return valid;
}

void uphip_align_mask(UphipImage image0, const UphipRectangle inside_area,
                      const UphipRectangle outside, UphipMaskAlignmentParameters params) {
  // align_mask_cpu, masks.c:265-300
  if (!ok_image(image0, "align_mask")) return;
  MonoProxy mp(image0, true, "align_mask");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return;
  const UphipImage image = mp.image();
  const Rect in = to_rect(inside_area), out = to_rect(outside);
  const int32_t iw = iabs(in.x0 - in.x1) + 1, ih = iabs(in.y0 - in.y1) + 1;
  int32_t tx, ty;
  if (params.alignment.left) tx = out.x0 + params.margin.horizontal;
  else if (params.alignment.right) tx = out.x1 - iw - params.margin.horizontal;
  else tx = (out.x0 + out.x1 - iw) / 2;
  if (params.alignment.top) ty = out.y0 + params.margin.vertical;
  else if (params.alignment.bottom) ty = out.y1 - ih - params.margin.vertical;
  else ty = (out.y0 + out.y1 - ih) / 2;
  UphipFrame* f = image.frame;
  MoveArgs a{in, tx, ty, {image.background.r, image.background.g, image.background.b}, 1};
  hipStream_t st = current_stream();
  UphipFrame* n = frame_alloc(f->width, f->height, f->format);
  if (!n) return;
  MoveArgs* d = stage_args(&a, 1, st);
  if (!d) return;
  launch_move_rect(ref_of(f), ref_of(n), d, 1, st);
  arg_fence(st);
  adopt_storage(f, n);
  mp.finish();
}

UphipBorder uphip_detect_border(UphipImage image0, UphipBorderScanParameters params,
                                const UphipRectangle outside_mask) {
  // detect_border_cpu / detect_border_edge, masks.c:410-488
  UphipBorder b{0, 0, 0, 0};
  if (!ok_image(image0, "detect_border")) return b;
  MonoProxy mp(image0, false, "detect_border");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return b;
  const UphipImage image = mp.image();
  UphipFrame* f = image.frame;
  const int32_t W = f->width, H = f->height;
  const Rect o = to_rect(outside_mask);
  b = UphipBorder{o.x0, o.y0, W - o.x1, H - o.y1};
  hipStream_t st = current_stream();
  const int32_t stride = imax(W, H);
  uint32_t* sums = (uint32_t*)scratch(0, sizeof(uint32_t) * stride * 2);
  int32_t* res = (int32_t*)scratch(1, sizeof(int32_t) * 4);
  if (!sums || !res) return b;
  UPH_HIP(hipMemsetAsync(sums, 0, sizeof(uint32_t) * stride * 2, st));
  const int32_t mw = iabs(o.x0 - o.x1) + 1, mh = iabs(o.y0 - o.y1) + 1;
  BorderEdgeArgs e[4];
  memset(e, 0, sizeof(e));
  if (params.scan_direction.horizontal) {
    // columns; the scanned rows are [o.y0, o.y1] as given (inverted = none)
    AxisArgs aa{clip(Rect{0, o.y0, W - 1, o.y1}, W, H), image.abs_black_threshold,
                o.y0 <= o.y1 ? 1 : 0};
    AxisArgs* d = stage_args(&aa, 1, st);
    if (!d) return b;
    if (aa.active && aa.region.y1 >= aa.region.y0)
      launch_axis_reduce(ref_of(f), d, 0, M_DARK_COUNT, W, H, sums, 0, 1, st);
    const int32_t sz = params.scan_size.width, stp = params.scan_step.horizontal;
    e[0] = BorderEdgeArgs{1, 0, W, o.x0, o.x0 + sz, stp, mw, params.scan_threshold.horizontal};
    e[1] = BorderEdgeArgs{1, 0, W, o.x1 - sz, o.x1, -stp, mw, params.scan_threshold.horizontal};
  }
  if (params.scan_direction.vertical) {
    AxisArgs aa{clip(Rect{o.x0, 0, o.x1, H - 1}, W, H), image.abs_black_threshold,
                o.x0 <= o.x1 ? 1 : 0};
    AxisArgs* d = stage_args(&aa, 1, st);
    if (!d) return b;
    if (aa.active && aa.region.x1 >= aa.region.x0)
      launch_axis_reduce(ref_of(f), d, 1, M_DARK_COUNT, W, H, sums + stride, 0, 1, st);
    const int32_t sz = params.scan_size.height, stp = params.scan_step.vertical;
    e[2] = BorderEdgeArgs{1, stride, H, o.y0, o.y0 + sz, stp, mh, params.scan_threshold.vertical};
    e[3] = BorderEdgeArgs{1, stride, H, o.y1 - sz, o.y1, -stp, mh, params.scan_threshold.vertical};
  }
  BorderEdgeArgs* de = stage_args(e, 4, st);
  if (!de) return b;
  UPH_HIP(hipMemsetAsync(res, 0, sizeof(int32_t) * 4, st));
  launch_border_scan(de, 4, sums, 0, res, 1, st, imax(W, H));
  arg_fence(st);
  int32_t r[4];
  UPH_HIP(hipMemcpyAsync(r, res, sizeof(r), hipMemcpyDeviceToHost, st));
  if (!UPH_HIP(hipStreamSynchronize(st))) return b;
  if (params.scan_direction.horizontal) {
    b.left += r[0];
    b.right += r[1];
  }
  if (params.scan_direction.vertical) {
    b.top += r[2];
    b.bottom += r[3];
  }
  return b;
}

// ---------------------------------------------------------------------------
// deskew.c peers
// ---------------------------------------------------------------------------
void uphip_deskew(UphipImage source0, UphipRectangle mask, float radians,
                  UphipInterpolation interp) {
  // deskew_cpu, deskew.c:272-286 (sin/cos of -radians with the host libm,
  // exactly as the reference computes them, deskew.c:260-261)
  if (!ok_image(source0, "deskew")) return;
  MonoProxy mp(source0, true, "deskew");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return;
  const UphipImage source = mp.image();
  UphipFrame* f = source.frame;
  RotateArgs a{to_rect(mask), sinf(-radians), cosf(-radians), 1};
  hipStream_t st = current_stream();
  UphipFrame* n = frame_alloc(f->width, f->height, f->format);
  if (!n) return;
  RotateArgs* d = stage_args(&a, 1, st);
  if (!d) return;
  if (!(interp == UPHIP_INTERP_LINEAR &&
        launch_rotate_linear(ref_of(f), ref_of(n), d, 1, 1, nullptr, 1, st, radians)))
    launch_rotate_mask(ref_of(f), ref_of(n), d, interp, 1, st, radians);
  arg_fence(st);
  adopt_storage(f, n);
  mp.finish();
}

}  // extern "C"
