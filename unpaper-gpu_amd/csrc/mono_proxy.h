// mono_proxy.h — 1-bit frames through the byte-format ops.
//
// The reference reads a MONOWHITE/MONOBLACK pixel as gray 0 or 255 and
// writes one by thresholding its gray value against the image's
// abs_black_threshold (pixel.c get_pixel/set_pixel).  The filter, detection
// and deskew kernels work on byte planes, so a 1-bit frame goes through them
// as a GRAY8 proxy holding exactly those 0/255 values; ops that write pack
// the proxy back with the same threshold.  Pixels an op leaves alone
// round-trip unchanged (0 < thr <= 255 keeps black black, 255 is never
// < thr), so the result equals the reference's per-pixel get/set on the
// 1-bit frame.  abs_black_threshold 0 cannot represent black on the way back
// and is refused.
#pragma once

#include "kernels.h"
#include "runtime.h"

namespace uph {

void launch_copy_thr(const PlaneRef& src, const PlaneRef& dst, const CopyArgs* args, int count,
                     int rows_hint, uint8_t thr, hipStream_t st);

class MonoProxy {
 public:
  MonoProxy(const UphipImage& im, bool writes, const char* op) : orig_(im), writes_(writes) {
    if (!im.frame || !is_mono(im.frame->format)) {
      ok_ = im.frame != nullptr;
      return;
    }
    if (im.abs_black_threshold == 0) {
      fail("%s: 1-bit frames need abs_black_threshold >= 1", op);
      return;
    }
    proxy_ = im;
    proxy_.frame = frame_alloc(im.frame->width, im.frame->height, F_GRAY8);
    if (!proxy_.frame) return;
    ok_ = convert(im.frame, proxy_.frame, im.abs_black_threshold);
  }
  ~MonoProxy() {
    if (proxy_.frame) frame_free(proxy_.frame);
  }
  MonoProxy(const MonoProxy&) = delete;
  MonoProxy& operator=(const MonoProxy&) = delete;

  bool ok() const { return ok_; }
  // the frame the op works on
  UphipImage image() const { return proxy_.frame ? proxy_ : orig_; }
  // write the op's result back into the 1-bit frame
  void finish() {
    if (proxy_.frame && writes_ && ok_) convert(proxy_.frame, orig_.frame, orig_.abs_black_threshold);
  }

 private:
  static bool convert(const UphipFrame* src, UphipFrame* dst, uint8_t thr) {
    hipStream_t st = current_stream();
    CopyArgs a{Rect{0, 0, src->width - 1, src->height - 1}, 0, 0, 1};
    CopyArgs* d = stage_args(&a, 1, st);
    if (!d) return false;
    launch_copy_thr(fixed_ref(frame_planes(src), 0), fixed_ref(frame_planes(dst), 0), d, 1,
                    src->height, thr, st);
    arg_fence(st);
    return true;
  }
  UphipImage orig_;
  UphipImage proxy_{nullptr, {255, 255, 255}, 0};
  bool writes_ = false;
  bool ok_ = false;
};

}  // namespace uph
