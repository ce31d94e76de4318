// interp.h — device restatement of imageprocess/interpolate.c.  Compiled with
// -ffp-contract=off and no fast-math so every float operation rounds exactly
// like the reference's scalar x86-64 code (same expression trees, same
// association order, IEEE add/mul/div).
#pragma once

#include "common.h"

namespace uph {

template <int FMT>
struct Src {
  const uint8_t* base;
  int64_t pitch;
  int32_t W, H;
  __device__ __forceinline__ Px at(int32_t x, int32_t y) const {
    if (x < 0 || y < 0 || x >= W || y >= H) return Px{255, 255, 255};
    return load_px_row<FMT>(base + (int64_t)y * pitch, x);
  }
};

// cubic_scale, interpolate.c:24-31 — identical expression.
__device__ __forceinline__ uint8_t cubic_scale(float factor, uint8_t a, uint8_t b, uint8_t c,
                                               uint8_t d) {
  int result = b + 0.5f * factor *
                       (c - a + factor * (2.0f * a - 5.0f * b + 4.0f * c - d +
                                          factor * (3.0f * (b - c) + d - a)));
  return (uint8_t)(result < 0 ? 0 : (result > 255 ? 255 : result));  // av_clip_uint8
}

__device__ __forceinline__ Px cubic_px(float f, Px a, Px b, Px c, Px d) {
  return Px{cubic_scale(f, a.r, b.r, c.r, d.r), cubic_scale(f, a.g, b.g, c.g, d.g),
            cubic_scale(f, a.b, b.b, c.b, d.b)};
}

// linear_scale, interpolate.c:62-65
__device__ __forceinline__ uint8_t linear_scale(float x, uint8_t a, uint8_t b) {
  return (uint8_t)((1.0f - x) * a + x * b);
}
__device__ __forceinline__ Px linear_px(float f, Px a, Px b) {
  return Px{linear_scale(f, a.r, b.r), linear_scale(f, a.g, b.g), linear_scale(f, a.b, b.b)};
}

// The interpolators are generic over the pixel source S (S::at(x, y) with
// get_pixel semantics): the global frame (Src) or an LDS-staged window.
template <class S>
__device__ __forceinline__ Px interp_nn(const S& s, float cx, float cy) {
  return s.at((int)roundf(cx), (int)roundf(cy));  // interpolate.c:13-18
}

template <class S>
__device__ __forceinline__ Px interp_bicubic(const S& s, float cx, float cy) {
  // interp_bicubic, interpolate.c:43-60: (int) truncates toward zero
  const int px = (int)cx, py = (int)cy;
  const float fx = cx - px;
  Px col[4];
#pragma unroll
  for (int i = -1; i < 3; ++i) {
    col[i + 1] = cubic_px(fx, s.at(px - 1, py + i), s.at(px, py + i), s.at(px + 1, py + i),
                          s.at(px + 2, py + i));
  }
  return cubic_px(cy - py, col[0], col[1], col[2], col[3]);
}

template <class S>
__device__ __forceinline__ Px interp_bilinear(const S& s, float cx, float cy) {
  // interp_bilinear, interpolate.c:77-118 (integral-coordinate quirk kept:
  // the one-axis cases use the OTHER axis' fraction, i.e. 0)
  const int x1 = (int)floorf(cx), y1 = (int)floorf(cy);
  const int x2 = (int)ceilf(cx), y2 = (int)ceilf(cy);
  if (!(x2 >= 0 && x2 <= s.W - 1 && y2 >= 0 && y2 <= s.H - 1)) return s.at(x1, y1);  // image size
  if (x1 == x2 && y1 == y2) return s.at(x1, y1);
  if (x1 == x2) return linear_px(cx - x1, s.at(x1, y1), s.at(x2, y2));
  if (y1 == y2) return linear_px(cy - y1, s.at(x1, y1), s.at(x2, y2));
  Px h1 = linear_px(cx - x1, s.at(x1, y1), s.at(x2, y1));
  Px h2 = linear_px(cx - x1, s.at(x1, y2), s.at(x2, y2));
  return linear_px(cy - y1, h1, h2);
}

template <int FMT, class S = Src<FMT>>
__device__ __forceinline__ Px interpolate(const S& s, float cx, float cy, int fn) {
  if (fn == UPHIP_INTERP_NN) return interp_nn(s, cx, cy);
  if (fn == UPHIP_INTERP_LINEAR) return interp_bilinear(s, cx, cy);
  return interp_bicubic(s, cx, cy);
}

}  // namespace uph
