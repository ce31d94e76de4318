// kernels_blit.hip — fill / copy / mask / geometry kernels (imageprocess/blit.c,
// masks.c apply/center/align, deskew.c rotate) for gfx950.
//
// All kernels are destination-driven: every output byte is produced by exactly
// one thread, so mono (1 bit per pixel) targets need no atomics (a thread owns
// a whole byte = 8 pixels).  Rows start 256-byte aligned, so the interior of a
// row is written with 16-byte stores.
#include <climits>
#include <type_traits>

#include "interp.h"
#include "kernels.h"

namespace uph {

constexpr int kThreads = 256;

// Write one pixel of any format into `row`; mono formats handled by callers.
__device__ __forceinline__ void store_px_fmt(uint8_t* row, int fmt, int32_t x, Px p) {
  if (fmt == F_GRAY8) store_px_row<F_GRAY8>(row, x, p);
  else if (fmt == F_Y400A) store_px_row<F_Y400A>(row, x, p);
  else store_px_row<F_RGB24>(row, x, p);
}

// Raw byte copy of one pixel (keeps Y400A alpha, as memcpy paths do).
template <int FMT>
__device__ __forceinline__ void copy_px_raw(uint8_t* drow, int32_t dx, const uint8_t* srow,
                                            int32_t sx) {
  constexpr int B = FMT == F_GRAY8 ? 1 : FMT == F_Y400A ? 2 : 3;
#pragma unroll
  for (int k = 0; k < B; k++) drow[dx * B + k] = srow[sx * B + k];
}

// set_pixel semantics for a mono byte: returns the new byte value after
// writing pixel bit `k` (0 = MSB) with colour p (pixel.c:142-168).
__device__ __forceinline__ uint8_t mono_set(uint8_t byte, int fmt, int k, Px p,
                                            uint8_t thr) {
  bool black = gray_of(p) < thr;
  if (fmt == F_MONOWHITE) black = !black;
  const uint8_t bit = (uint8_t)(128 >> k);
  return black ? (uint8_t)(byte & ~bit) : (uint8_t)(byte | bit);
}

// Uniform byte fill of [b0, b1) of a 16-byte aligned row.
__device__ __forceinline__ void fill_bytes(uint8_t* row, int64_t b0, int64_t b1, uint8_t v) {
  const int64_t c0 = b0 >> 4, c1 = (b1 + 15) >> 4;
  const uint32_t w = v * 0x01010101u;
  const uint4 q = make_uint4(w, w, w, w);
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
    const int64_t s = c << 4;
    if (s >= b0 && s + 16 <= b1) {
      *reinterpret_cast<uint4*>(row + s) = q;
    } else {
      for (int k = 0; k < 16; k++) {
        const int64_t b = s + k;
        if (b >= b0 && b < b1) row[b] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// wipe_rectangle_cpu (blit.c:20-24): args[s].r is already clipped.
// ---------------------------------------------------------------------------
struct FillLaunch {
  PlaneRef dst;
  const FillArgs* args;
  uint8_t thr;
};

__global__ void __launch_bounds__(kThreads) k_fill(FillLaunch L) {
  const int s = blockIdx.z;
  const FillArgs a = L.args[s];
  if (!a.active || a.r.x1 < a.r.x0 || a.r.y1 < a.r.y0) return;
  const Planes& P = L.dst.P;
  uint8_t* base = plane_ptr(L.dst, s);
  const Px c{a.color[0], a.color[1], a.color[2]};
  for (int32_t y = a.r.y0 + blockIdx.x; y <= a.r.y1; y += gridDim.x) {
    uint8_t* row = base + (int64_t)y * P.pitch;
    if (P.fmt == F_GRAY8) {
      fill_bytes(row, a.r.x0, (int64_t)a.r.x1 + 1, gray_of(c));
    } else if (P.fmt == F_RGB24 && c.r == c.g && c.g == c.b) {
      fill_bytes(row, 3 * (int64_t)a.r.x0, 3 * ((int64_t)a.r.x1 + 1), c.r);
    } else if (P.fmt == F_RGB24 || P.fmt == F_Y400A) {
      for (int32_t x = a.r.x0 + threadIdx.x; x <= a.r.x1; x += blockDim.x)
        store_px_fmt(row, P.fmt, x, c);
    } else {  // mono: one thread per byte
      const int32_t b0 = a.r.x0 >> 3, b1 = a.r.x1 >> 3;
      for (int32_t b = b0 + threadIdx.x; b <= b1; b += blockDim.x) {
        uint8_t v = row[b];
        for (int k = 0; k < 8; k++) {
          const int32_t x = b * 8 + k;
          if (x >= a.r.x0 && x <= a.r.x1) v = mono_set(v, P.fmt, k, c, L.thr);
        }
        row[b] = v;
      }
    }
  }
}

void launch_fill(const PlaneRef& dst, const FillArgs* args, int count, int rows_hint,
                 hipStream_t st) {
  FillLaunch L{dst, args, 0};
  int gx = rows_hint < 1 ? 1 : (rows_hint > 1024 ? 1024 : rows_hint);
  hipLaunchKernelGGL(k_fill, dim3(gx, 1, count), dim3(kThreads), 0, st, L);
}

// Mono-aware fill (needs the frame's abs_black_threshold).
void launch_fill_thr(const PlaneRef& dst, const FillArgs* args, int count, int rows_hint,
                     uint8_t thr, hipStream_t st) {
  FillLaunch L{dst, args, thr};
  int gx = rows_hint < 1 ? 1 : (rows_hint > 1024 ? 1024 : rows_hint);
  hipLaunchKernelGGL(k_fill, dim3(gx, 1, count), dim3(kThreads), 0, st, L);
}

// ---------------------------------------------------------------------------
// copy_rectangle_cpu (blit.c:30-80): dst(tx+u, ty+v) = src(a.x0+u, a.y0+v)
// for (u,v) in the clipped source area; target writes outside are dropped.
// Format conversion goes through get_pixel/set_pixel semantics.
// ---------------------------------------------------------------------------
struct CopyLaunch {
  PlaneRef src, dst;
  const CopyArgs* args;
  uint8_t thr;  // target abs_black_threshold (mono targets)
};

__global__ void __launch_bounds__(kThreads) k_copy(CopyLaunch L) {
  const int s = blockIdx.z;
  const CopyArgs a = L.args[s];
  if (!a.active || a.a.x1 < a.a.x0 || a.a.y1 < a.a.y0) return;
  const Planes& S = L.src.P;
  const Planes& D = L.dst.P;
  const uint8_t* sbase = plane_ptr(L.src, s);
  uint8_t* dbase = plane_ptr(L.dst, s);
  // target columns covered: [tx, tx + w) ∩ [0, D.W)
  const int32_t w = a.a.x1 - a.a.x0 + 1;
  const int32_t tx0 = imax(a.tx, 0), tx1 = imin(a.tx + w - 1, D.W - 1);
  if (tx1 < tx0) return;
  const int32_t h = a.a.y1 - a.a.y0 + 1;
  // blit.c:38-69: the memcpy path (raw bytes, Y400A alpha kept) is taken only
  // when the whole target rectangle lies inside the target frame; otherwise
  // set_pixel per pixel (Y400A alpha := 0xFF).  Identical for GRAY8/RGB24.
  const bool fully_inside = a.tx >= 0 && a.ty >= 0 && a.tx + w <= D.W && a.ty + h <= D.H;
  const bool same_bytes =
      S.fmt == D.fmt && !is_mono(S.fmt) && (fully_inside || S.fmt != F_Y400A);
  const int bpp = bytes_per_pixel(D.fmt);
  for (int32_t sy = a.a.y0 + blockIdx.x; sy <= a.a.y1; sy += gridDim.x) {
    const int32_t ty = a.ty + (sy - a.a.y0);
    if (ty < 0 || ty >= D.H) continue;
    const uint8_t* srow = sbase + (int64_t)sy * S.pitch;
    uint8_t* drow = dbase + (int64_t)ty * D.pitch;
    if (same_bytes) {
      // byte copy: dst bytes [tx0*bpp, (tx1+1)*bpp) from src shifted by delta
      const int64_t db0 = (int64_t)tx0 * bpp, db1 = ((int64_t)tx1 + 1) * bpp;
      const int64_t delta = ((int64_t)a.a.x0 - a.tx) * bpp;  // src byte = dst byte + delta
      // 16-byte vectors when source and target rows share their alignment
      // (pages read in place may come with any pitch)
      if ((delta & 15) == 0 && (((uintptr_t)srow - (uintptr_t)drow) & 15) == 0) {
        const int64_t c0 = db0 >> 4, c1 = (db1 + 15) >> 4;
        for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
          const int64_t b = c << 4;
          if (b >= db0 && b + 16 <= db1) {
            *reinterpret_cast<uint4*>(drow + b) =
                *reinterpret_cast<const uint4*>(srow + b + delta);
          } else {
            for (int k = 0; k < 16; k++)
              if (b + k >= db0 && b + k < db1) drow[b + k] = srow[b + k + delta];
          }
        }
      } else {
        for (int64_t b = db0 + threadIdx.x; b < db1; b += blockDim.x) drow[b] = srow[b + delta];
      }
    } else if (!is_mono(D.fmt)) {
      for (int32_t tx = tx0 + threadIdx.x; tx <= tx1; tx += blockDim.x) {
        const int32_t sx = a.a.x0 + (tx - a.tx);
        store_px_fmt(drow, D.fmt, tx,
                     load_px_any(sbase, S.pitch, S.fmt, S.W, S.H, sx, sy));
      }
    } else {
      for (int32_t b = (tx0 >> 3) + threadIdx.x; b <= (tx1 >> 3); b += blockDim.x) {
        uint8_t v = drow[b];
        for (int k = 0; k < 8; k++) {
          const int32_t tx = b * 8 + k;
          if (tx < tx0 || tx > tx1) continue;
          const int32_t sx = a.a.x0 + (tx - a.tx);
          v = mono_set(v, D.fmt, k, load_px_any(sbase, S.pitch, S.fmt, S.W, S.H, sx, sy), L.thr);
        }
        drow[b] = v;
      }
    }
  }
}

void launch_copy_thr(const PlaneRef& src, const PlaneRef& dst, const CopyArgs* args, int count,
                     int rows_hint, uint8_t thr, hipStream_t st) {
  CopyLaunch L{src, dst, args, thr};
  int gx = rows_hint < 1 ? 1 : (rows_hint > 1024 ? 1024 : rows_hint);
  UPH_LAUNCH_DIAG(8, k_copy, dim3(gx, 1, count), dim3(kThreads), 0, st, L);
}

void launch_copy(const PlaneRef& src, const PlaneRef& dst, const CopyArgs* args, int count,
                 int rows_hint, hipStream_t st) {
  launch_copy_thr(src, dst, args, count, rows_hint, 0, st);
}

// ---------------------------------------------------------------------------
// apply_masks_cpu (masks.c:306-322): pixels outside every mask <- colour.
// No reads of the image: outside pixels are written, inside left untouched.
// ---------------------------------------------------------------------------
struct MasksLaunch {
  PlaneRef dst;
  const MaskArgs* args;
  uint8_t thr;
};

__global__ void __launch_bounds__(kThreads) k_apply_masks(MasksLaunch L) {
  const int s = blockIdx.z;
  const MaskArgs* a = L.args + s;
  const int32_t n = a->n;
  if (n <= 0) return;
  __shared__ Rect m[UPHIP_MAX_MASKS];
  for (int i = threadIdx.x; i < n; i += blockDim.x) m[i] = normalize(a->m[i]);
  __syncthreads();
  const Planes& P = L.dst.P;
  uint8_t* base = plane_ptr(L.dst, s);
  const Px c{a->color[0], a->color[1], a->color[2]};
  if (n == 1 && P.fmt == F_GRAY8) {
    // one mask on a gray plane: every row is at most two runs outside it,
    // written with 16-byte stores
    const Rect m0 = m[0];
    const uint8_t v = gray_of(c);
    for (int32_t y = blockIdx.x; y < P.H; y += gridDim.x) {
      uint8_t* row = base + (int64_t)y * P.pitch;
      if (y < m0.y0 || y > m0.y1 || m0.x1 < 0 || m0.x0 >= P.W) {
        fill_bytes(row, 0, P.W, v);
      } else {
        if (m0.x0 > 0) fill_bytes(row, 0, imin(m0.x0, P.W), v);
        if (m0.x1 < P.W - 1) fill_bytes(row, imax(m0.x1 + 1, 0), P.W, v);
      }
    }
    return;
  }
  for (int32_t y = blockIdx.x; y < P.H; y += gridDim.x) {
    uint8_t* row = base + (int64_t)y * P.pitch;
    if (!is_mono(P.fmt)) {
      for (int32_t x = threadIdx.x; x < P.W; x += blockDim.x) {
        bool inside = false;
        for (int i = 0; i < n && !inside; i++)
          inside = x >= m[i].x0 && x <= m[i].x1 && y >= m[i].y0 && y <= m[i].y1;
        if (!inside) store_px_fmt(row, P.fmt, x, c);
      }
    } else {
      for (int32_t b = threadIdx.x; b < (P.W + 7) / 8; b += blockDim.x) {
        uint8_t v = row[b];
        for (int k = 0; k < 8; k++) {
          const int32_t x = b * 8 + k;
          if (x >= P.W) break;
          bool inside = false;
          for (int i = 0; i < n && !inside; i++)
            inside = x >= m[i].x0 && x <= m[i].x1 && y >= m[i].y0 && y <= m[i].y1;
          if (!inside) v = mono_set(v, P.fmt, k, c, L.thr);
        }
        row[b] = v;
      }
    }
  }
}

void launch_apply_masks_thr(const PlaneRef& dst, const MaskArgs* args, int count, uint8_t thr,
                            hipStream_t st) {
  MasksLaunch L{dst, args, thr};
  int gx = dst.P.H < 1 ? 1 : (dst.P.H > 1024 ? 1024 : dst.P.H);
  hipLaunchKernelGGL(k_apply_masks, dim3(gx, 1, count), dim3(kThreads), 0, st, L);
}
void launch_apply_masks(const PlaneRef& dst, const MaskArgs* args, int count, hipStream_t st) {
  launch_apply_masks_thr(dst, args, count, 0, st);
}

// ---------------------------------------------------------------------------
// Generic destination-driven gather: dst(x,y) = src(map(x,y)) or a constant.
// Used for mirror, rotate90, shift (out of place).
// ---------------------------------------------------------------------------
enum GatherKind : int32_t { G_MIRROR = 0, G_ROT90 = 1, G_SHIFT = 2 };

struct GatherLaunch {
  PlaneRef src, dst;
  int32_t kind;
  int32_t p0, p1;   // mirror: h, v; rot90: direction; shift: dx, dy
  uint8_t bg[3];
  uint8_t thr;
};

__device__ __forceinline__ Px gather_px(const GatherLaunch& L, const uint8_t* sbase, int32_t x,
                                        int32_t y) {
  const Planes& S = L.src.P;
  int32_t sx, sy;
  if (L.kind == G_MIRROR) {
    sx = L.p0 ? S.W - 1 - x : x;
    sy = L.p1 ? S.H - 1 - y : y;
  } else if (L.kind == G_ROT90) {
    // flip_rotate_90_cpu (blit.c:289-310) inverted: dst(xx,yy) = src(x,y)
    if (L.p0 > 0) {  // xx = H-1-y, yy = x
      sx = y;
      sy = S.H - 1 - x;
    } else {         // xx = y, yy = W-1-x
      sx = S.W - 1 - y;
      sy = x;
    }
  } else {  // shift: new frame filled with background, src copied at (dx,dy)
    sx = x - L.p0;
    sy = y - L.p1;
    if (sx < 0 || sy < 0 || sx >= S.W || sy >= S.H) return Px{L.bg[0], L.bg[1], L.bg[2]};
  }
  return load_px_any(sbase, S.pitch, S.fmt, S.W, S.H, sx, sy);
}

__global__ void __launch_bounds__(kThreads) k_gather(GatherLaunch L) {
  const int s = blockIdx.z;
  const Planes& D = L.dst.P;
  const uint8_t* sbase = plane_ptr(L.src, s);
  uint8_t* dbase = plane_ptr(L.dst, s);
  for (int32_t y = blockIdx.x; y < D.H; y += gridDim.x) {
    uint8_t* row = dbase + (int64_t)y * D.pitch;
    if (!is_mono(D.fmt)) {
      for (int32_t x = threadIdx.x; x < D.W; x += blockDim.x)
        store_px_fmt(row, D.fmt, x, gather_px(L, sbase, x, y));
    } else {
      for (int32_t b = threadIdx.x; b < (D.W + 7) / 8; b += blockDim.x) {
        uint8_t v = row[b];
        for (int k = 0; k < 8; k++) {
          const int32_t x = b * 8 + k;
          if (x >= D.W) break;
          v = mono_set(v, D.fmt, k, gather_px(L, sbase, x, y), L.thr);
        }
        row[b] = v;
      }
    }
  }
}

static void launch_gather(const GatherLaunch& L, int count, hipStream_t st) {
  int gx = L.dst.P.H < 1 ? 1 : (L.dst.P.H > 1024 ? 1024 : L.dst.P.H);
  hipLaunchKernelGGL(k_gather, dim3(gx, 1, count), dim3(kThreads), 0, st, L);
}

void launch_mirror_oop(const PlaneRef& src, const PlaneRef& dst, bool h, bool v, uint8_t thr,
                       int count, hipStream_t st) {
  GatherLaunch L{src, dst, G_MIRROR, h ? 1 : 0, v ? 1 : 0, {0, 0, 0}, thr};
  launch_gather(L, count, st);
}
void launch_rotate90_thr(const PlaneRef& src, const PlaneRef& dst, int direction, uint8_t thr,
                         int count, hipStream_t st) {
  GatherLaunch L{src, dst, G_ROT90, direction, 0, {0, 0, 0}, thr};
  launch_gather(L, count, st);
}
void launch_rotate90(const PlaneRef& src, const PlaneRef& dst, int direction, int count,
                     hipStream_t st) {
  launch_rotate90_thr(src, dst, direction, 0, count, st);
}
void launch_shift(const PlaneRef& src, const PlaneRef& dst, int dx, int dy, const uint8_t bg[3],
                  uint8_t thr, int count, hipStream_t st) {
  GatherLaunch L{src, dst, G_SHIFT, dx, dy, {bg[0], bg[1], bg[2]}, thr};
  launch_gather(L, count, st);
}
void launch_mirror(const PlaneRef&, bool, bool, int, hipStream_t) {}

// ---------------------------------------------------------------------------
// stretch_frame (blit.c:209-229): dst(x,y) = interpolate(src, x*hr, y*vr).
// ---------------------------------------------------------------------------
struct StretchLaunch {
  PlaneRef src, dst;
  int32_t interp;
  float hr, vr;
  uint8_t thr;
};

template <int SF>
__device__ __forceinline__ Px stretch_px(const StretchLaunch& L, const uint8_t* sbase, int32_t x,
                                         int32_t y) {
  Src<SF> s{sbase, L.src.P.pitch, L.src.P.W, L.src.P.H};
  return interpolate<SF>(s, x * L.hr, y * L.vr, L.interp);
}

__device__ __forceinline__ Px stretch_any(const StretchLaunch& L, const uint8_t* sbase, int32_t x,
                                          int32_t y) {
  switch (L.src.P.fmt) {
    case F_GRAY8: return stretch_px<F_GRAY8>(L, sbase, x, y);
    case F_Y400A: return stretch_px<F_Y400A>(L, sbase, x, y);
    case F_RGB24: return stretch_px<F_RGB24>(L, sbase, x, y);
    default: {
      // mono sources: interpolate over the 0/255 expansion
      const Planes& S = L.src.P;
      struct MonoSrc {
        const uint8_t* b;
        int64_t p;
        int f;
        int32_t W, H;
      } ms{sbase, S.pitch, S.fmt, S.W, S.H};
      (void)ms;
      // NN / linear / cubic on a mono source read through load_px_any
      const float cx = x * L.hr, cy = y * L.vr;
      auto at = [&](int32_t xx, int32_t yy) {
        return load_px_any(sbase, S.pitch, S.fmt, S.W, S.H, xx, yy);
      };
      if (L.interp == UPHIP_INTERP_NN) return at((int)roundf(cx), (int)roundf(cy));
      if (L.interp == UPHIP_INTERP_LINEAR) {
        const int x1 = (int)floorf(cx), y1 = (int)floorf(cy);
        const int x2 = (int)ceilf(cx), y2 = (int)ceilf(cy);
        if (!(x2 >= 0 && x2 <= S.W - 1 && y2 >= 0 && y2 <= S.H - 1)) return at(x1, y1);
        if (x1 == x2 && y1 == y2) return at(x1, y1);
        if (x1 == x2) return linear_px(cx - x1, at(x1, y1), at(x2, y2));
        if (y1 == y2) return linear_px(cy - y1, at(x1, y1), at(x2, y2));
        Px h1 = linear_px(cx - x1, at(x1, y1), at(x2, y1));
        Px h2 = linear_px(cx - x1, at(x1, y2), at(x2, y2));
        return linear_px(cy - y1, h1, h2);
      }
      const int px = (int)cx, py = (int)cy;
      Px col[4];
      for (int i = -1; i < 3; ++i)
        col[i + 1] = cubic_px(cx - px, at(px - 1, py + i), at(px, py + i), at(px + 1, py + i),
                              at(px + 2, py + i));
      return cubic_px(cy - py, col[0], col[1], col[2], col[3]);
    }
  }
}

__global__ void __launch_bounds__(kThreads) k_stretch(StretchLaunch L) {
  const int s = blockIdx.z;
  const Planes& D = L.dst.P;
  const uint8_t* sbase = plane_ptr(L.src, s);
  uint8_t* dbase = plane_ptr(L.dst, s);
  for (int32_t y = blockIdx.x; y < D.H; y += gridDim.x) {
    uint8_t* row = dbase + (int64_t)y * D.pitch;
    if (!is_mono(D.fmt)) {
      for (int32_t x = threadIdx.x; x < D.W; x += blockDim.x)
        store_px_fmt(row, D.fmt, x, stretch_any(L, sbase, x, y));
    } else {
      for (int32_t b = threadIdx.x; b < (D.W + 7) / 8; b += blockDim.x) {
        uint8_t v = row[b];
        for (int k = 0; k < 8; k++) {
          const int32_t x = b * 8 + k;
          if (x >= D.W) break;
          v = mono_set(v, D.fmt, k, stretch_any(L, sbase, x, y), L.thr);
        }
        row[b] = v;
      }
    }
  }
}

void launch_stretch_thr(const PlaneRef& src, const PlaneRef& dst, int interp, uint8_t thr,
                        int count, hipStream_t st) {
  StretchLaunch L{src, dst, interp, (float)src.P.W / (float)dst.P.W,
                  (float)src.P.H / (float)dst.P.H, thr};
  int gx = dst.P.H < 1 ? 1 : (dst.P.H > 1024 ? 1024 : dst.P.H);
  hipLaunchKernelGGL(k_stretch, dim3(gx, 1, count), dim3(kThreads), 0, st, L);
}
void launch_stretch(const PlaneRef& src, const PlaneRef& dst, int interp, int count,
                    hipStream_t st) {
  launch_stretch_thr(src, dst, interp, 0, count, st);
}

// ---------------------------------------------------------------------------
// center_mask / align_mask as a single out-of-place gather (masks.c:222-300):
//   newimage = bg-filled |area|; copy clip(area) -> newimage at (0,0);
//   wipe clip(area) with bg; copy newimage -> image at (tx,ty).
// ---------------------------------------------------------------------------
template <int FMT>
__global__ void __launch_bounds__(kThreads) k_move_rect(PlaneRef src, PlaneRef dst,
                                                        const MoveArgs* args) {
  const int s = blockIdx.z;
  const MoveArgs a = args[s];
  if (!a.active) return;
  const Planes& P = src.P;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const Rect A = clip(a.area, P.W, P.H);
  const int32_t aw = A.x1 - A.x0 + 1, ah = A.y1 - A.y0 + 1;  // copied extent (may be <= 0)
  const int32_t sw = iabs(a.area.x0 - a.area.x1) + 1, sh = iabs(a.area.y0 - a.area.y1) + 1;
  const Px bg{a.bg[0], a.bg[1], a.bg[2]};
  // the paste back (copy_rectangle newimage -> image) is a raw memcpy only when
  // the whole target rectangle is inside the image (blit.c:38-69); otherwise
  // set_pixel per pixel, which rewrites Y400A alpha as 0xFF
  const bool raw_paste = a.tx >= 0 && a.ty >= 0 && a.tx + sw <= P.W && a.ty + sh <= P.H;
  for (int32_t y = blockIdx.x; y < P.H; y += gridDim.x) {
    const uint8_t* srow = sbase + (int64_t)y * P.pitch;
    uint8_t* drow = dbase + (int64_t)y * P.pitch;
    const int32_t v = y - a.ty;
    for (int32_t x = threadIdx.x; x < P.W; x += blockDim.x) {
      const int32_t u = x - a.tx;
      Px o;
      if (u >= 0 && u < sw && v >= 0 && v < sh) {
        if (u < aw && v < ah) {
          const uint8_t* srow_m = sbase + (int64_t)(A.y0 + v) * P.pitch;
          if (raw_paste) {
            copy_px_raw<FMT>(drow, x, srow_m, A.x0 + u);
            continue;
          }
          o = load_px_row<FMT>(srow_m, A.x0 + u);
        } else {
          o = bg;
        }
      } else if (x >= A.x0 && x <= A.x1 && y >= A.y0 && y <= A.y1) {
        o = bg;
      } else {
        copy_px_raw<FMT>(drow, x, srow, x);
        continue;
      }
      store_px_row<FMT>(drow, x, o);
    }
  }
}

// k_move_rect for RGB24 planes, a destination dword per lane.  A moved
// pixel's bytes come from the same row offset 3 (A.x0 - tx) away, so a dword
// whose bytes all share one class (unchanged / background / moved) is one
// aligned load, a constant pattern, or two aligned loads realigned by that
// offset; dwords across a class change, and the row's tail, go byte by byte.
// RGB24 has no alpha: set_pixel and the raw paste write the same bytes.
__global__ void __launch_bounds__(kThreads) k_move_rect_rgb(PlaneRef src, PlaneRef dst,
                                                            const MoveArgs* args) {
  const int s = blockIdx.z;
  const MoveArgs a = args[s];
  if (!a.active) return;
  const Planes& P = src.P;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const Rect A = clip(a.area, P.W, P.H);
  const int32_t aw = A.x1 - A.x0 + 1, ah = A.y1 - A.y0 + 1;
  const int32_t sw = iabs(a.area.x0 - a.area.x1) + 1, sh = iabs(a.area.y0 - a.area.y1) + 1;
  const int32_t rowb = 3 * P.W, ndw = (rowb + 3) >> 2;
  const int32_t shift = 3 * (A.x0 - a.tx);  // source byte - destination byte, moved pixels
  // the background as bytes of a dword starting at a byte of phase 0, 1, 2
  uint32_t bgw[3];
#pragma unroll
  for (int ph = 0; ph < 3; ph++) {
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) w |= (uint32_t)a.bg[(ph + k) % 3] << (8 * k);
    bgw[ph] = w;
  }
  for (int32_t y = blockIdx.x; y < P.H; y += gridDim.x) {
    const uint8_t* srow = sbase + (int64_t)y * P.pitch;
    uint8_t* drow = dbase + (int64_t)y * P.pitch;
    const int32_t v = y - a.ty;
    const bool vin = v >= 0 && v < sh, vsrc = vin && v < ah;
    const bool wrow = y >= A.y0 && y <= A.y1;
    const uint8_t* srow_m = sbase + (int64_t)(A.y0 + (vsrc ? v : 0)) * P.pitch;
    // 0 unchanged, 1 background, 2 moved
    auto cls = [&](int32_t x) {
      const int32_t u = x - a.tx;
      if (vin && u >= 0 && u < sw) return vsrc && u < aw ? 2 : 1;
      return wrow && x >= A.x0 && x <= A.x1 ? 1 : 0;
    };
    for (int32_t d = threadIdx.x; d < ndw; d += blockDim.x) {
      const int32_t xb = 4 * d;
      const int c0 = cls(xb / 3), c1 = cls(imin(xb + 3, rowb - 1) / 3);
      if (c0 == c1 && xb + 4 <= rowb) {
        uint32_t out;
        if (c0 == 0) {
          out = *reinterpret_cast<const uint32_t*>(srow + xb);
        } else if (c0 == 1) {
          out = bgw[xb % 3];
        } else {
          const int32_t sb = xb + shift, sa = sb & ~3, r = sb & 3;
          const uint32_t w0 = *reinterpret_cast<const uint32_t*>(srow_m + sa);
          out = r ? __builtin_amdgcn_alignbyte(*reinterpret_cast<const uint32_t*>(srow_m + sa + 4), w0, r)
                  : w0;
        }
        *reinterpret_cast<uint32_t*>(drow + xb) = out;
      } else {
        for (int k = 0; k < 4 && xb + k < rowb; k++) {
          const int32_t b = xb + k, x = b / 3, c = cls(x);
          drow[b] = c == 0 ? srow[b] : c == 1 ? a.bg[b % 3] : srow_m[b + shift];
        }
      }
    }
  }
}

// k_move_rect for gray planes, 16 bytes of the destination per lane.  The
// class of a column (unchanged / background / moved) only changes at five
// breakpoints, so a vector not straddling one is one aligned 16-byte load, a
// constant, or two aligned loads realigned by the source shift, which is the
// same for every vector of the sheet ((A.x0 - tx) mod 16).  Vectors across a
// breakpoint or the right image edge go byte by byte.
template <int Q>
__device__ __forceinline__ uint4 shift_bytes16(const uint32_t* w, int r) {
  return make_uint4(__builtin_amdgcn_alignbyte(w[Q + 1], w[Q], r),
                    __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], r),
                    __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], r),
                    __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], r));
}

constexpr int kMoveRows = 8;  // rows per wave of k_move_rect_g16
constexpr int kMoveBp = 7;    // column breakpoints: five of the move, two of a folded mask
constexpr int kMoveBlockRows = kMoveRows * (kThreads / 64);
static_assert((kMoveBp + 1) * kMoveBlockRows <= kThreads, "one lane per deferred (row, vector)");

// bytes <= thr among four (kadd = (256 - (thr + 1)) * 0x00010001), keeping
// the bytes whose bit is set in `keep4` (bits 0..3 = bytes 0..3)
__device__ __forceinline__ uint32_t dark4(uint32_t x, uint32_t kadd, uint32_t keep4) {
  const uint32_t lo = ((x & 0x00FF00FFu) + kadd) & 0x01000100u;  // bytes 0, 2 > thr: bits 8, 24
  const uint32_t hi = (((x >> 8) & 0x00FF00FFu) + kadd) & 0x01000100u;  // bytes 1, 3
  const uint32_t kb = ((keep4 & 1u) << 8) | ((keep4 & 2u) << 8) | ((keep4 & 4u) << 22) |
                      ((keep4 & 8u) << 22);  // keep bits at 8, 9, 24, 25
  return __popc(kb) - __popc((lo | (hi << 1)) & kb);
}
// dark bytes of a 16-byte vector, bytes selected by a 16-bit mask
__device__ __forceinline__ uint32_t dark16(const uint4& v, uint32_t m16, uint32_t kadd) {
  return dark4(v.x, kadd, m16 & 15u) + dark4(v.y, kadd, (m16 >> 4) & 15u) +
         dark4(v.z, kadd, (m16 >> 8) & 15u) + dark4(v.w, kadd, m16 >> 12);
}
// 16-bit mask of the columns x0 .. x0+15 inside [c0, c1]
__device__ __forceinline__ uint32_t cols16(int32_t x0, int32_t c0, int32_t c1) {
  const int32_t lo = imax(c0 - x0, 0), hi = imin(c1 - x0, 15);
  return lo > hi ? 0u : ((2u << hi) - 1u) & ~((1u << lo) - 1u);
}
// byte mask of the four bits b (bit j -> byte j)
__device__ __forceinline__ uint32_t bytes_of4(uint32_t b) {
  return ((b * 0x00204081u) & 0x01010101u) * 0xFFu;
}

template <int MODE>
__global__ void __launch_bounds__(kThreads) k_move_rect_g16(PlaneRef src, PlaneRef dst,
                                                            const MoveArgs* args, MoveExtra X) {
  constexpr bool kMask = (MODE & 1) != 0, kRows = (MODE & 2) != 0;
  constexpr bool kDry = (MODE & 4) != 0;  // count only: nothing is written
  static_assert(!(kDry && kMask), "a dry pass counts; it does not mask");
  const int s = blockIdx.z;
  if (X.only && !X.only[s]) return;
  const MoveArgs a = args[s];
  if (!kMask && !kRows && !a.active) return;
  const Planes& P = src.P;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const int lane = threadIdx.x & 63;
  const int32_t nv = (P.W + 15) >> 4;                  // vectors per row (inside the pitch)
  // the block's rows: blocks cover the row ranges [ya0, ya1) then [yb0, yb1)
  // (all rows by default), kMoveBlockRows each
  const bool ranged = X.ya1 > X.ya0 || X.yb1 > X.yb0;
  const int32_t ra0 = ranged ? X.ya0 : 0, ra1 = ranged ? X.ya1 : P.H;
  const int32_t nba = ra1 > ra0 ? (ra1 - ra0 + kMoveBlockRows - 1) / kMoveBlockRows : 0;
  const bool second = (int32_t)blockIdx.x >= nba;
  const int32_t yb = second ? X.yb0 + ((int32_t)blockIdx.x - nba) * kMoveBlockRows
                            : ra0 + (int32_t)blockIdx.x * kMoveBlockRows;  // the block's first row
  const int32_t yend = imin(second ? X.yb1 : ra1, P.H);  // first row past the block's range
  const int32_t y0 = yb + (threadIdx.x >> 6) * kMoveRows;
  const int32_t y1 = imin(y0 + kMoveRows, yend);
  // folded apply_masks (one mask, masks.c:306-322 semantics: normalized,
  // pixels outside it <- colour)
  Rect mk{INT_MIN / 2, INT_MIN / 2, INT_MAX / 2, INT_MAX / 2};
  uint8_t mcol = 0;
  if (kMask) {
    const MaskArgs* ma = X.masks + s;
    if (ma->n > 0) mk = normalize(ma->m[0]);
    mcol = gray_of(Px{ma->color[0], ma->color[1], ma->color[2]});
  }
  const uint32_t mcol4 = mcol * 0x01010101u;
  const uint32_t kadd = (256u - ((uint32_t)X.thr + 1u)) * 0x00010001u;
  __shared__ uint32_t rowcnt[kMoveBlockRows];
  if (kRows) {
    if (threadIdx.x < kMoveBlockRows) rowcnt[threadIdx.x] = 0;
    __syncthreads();
  }
  uint32_t acc[kMoveRows];
#pragma unroll
  for (int k = 0; k < kMoveRows; k++) acc[k] = 0;
  auto finish_rows = [&]() {
    if (!kRows) return;
#pragma unroll
    for (int k = 0; k < kMoveRows; k++) {
      uint32_t v = acc[k];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane == 0 && v) atomicAdd(&rowcnt[y0 - yb + k], v);
    }
    __syncthreads();
    const int32_t y = yb + (int32_t)threadIdx.x;
    if (threadIdx.x < kMoveBlockRows && y < yend) X.rows[(int64_t)s * X.rows_stride + y] = rowcnt[threadIdx.x];
  };
  if (!a.active) {
    // the identity move: mask the current plane in place and/or count it
    for (int32_t vi = lane; vi < nv; vi += 64) {
      const int32_t x0 = 16 * vi;
      const uint32_t valid = cols16(x0, 0, P.W - 1);
      const uint32_t incol = cols16(x0, mk.x0, mk.x1) & valid;
      const uint32_t reg = kRows ? cols16(x0, X.rx0, X.rx1) : 0u;
#pragma unroll
      for (int k = 0; k < kMoveRows; k++) {
        const int32_t y = y0 + k;
        if (y >= y1) break;
        uint8_t* row = const_cast<uint8_t*>(sbase) + (int64_t)y * P.pitch;
        const uint32_t out16 = kMask ? valid & ~((y >= mk.y0 && y <= mk.y1) ? incol : 0u) : 0u;
        uint4 v = make_uint4(mcol4, mcol4, mcol4, mcol4);
        if ((kRows && reg) || out16 != valid || valid != 0xFFFFu)
          v = *reinterpret_cast<const uint4*>(row + x0);
        if (out16) {
          v.x = (v.x & ~bytes_of4(out16 & 15u)) | (mcol4 & bytes_of4(out16 & 15u));
          v.y = (v.y & ~bytes_of4((out16 >> 4) & 15u)) | (mcol4 & bytes_of4((out16 >> 4) & 15u));
          v.z = (v.z & ~bytes_of4((out16 >> 8) & 15u)) | (mcol4 & bytes_of4((out16 >> 8) & 15u));
          v.w = (v.w & ~bytes_of4(out16 >> 12)) | (mcol4 & bytes_of4(out16 >> 12));
          *reinterpret_cast<uint4*>(row + x0) = v;
        }
        if (kRows && reg) acc[k] += dark16(v, reg, kadd);
      }
    }
    finish_rows();
    return;
  }
  const Rect A = clip(a.area, P.W, P.H);
  const int32_t aw = A.x1 - A.x0 + 1, ah = A.y1 - A.y0 + 1;
  const int32_t sw = iabs(a.area.x0 - a.area.x1) + 1, sh = iabs(a.area.y0 - a.area.y1) + 1;
  const uint8_t bg = gray_of(Px{a.bg[0], a.bg[1], a.bg[2]});
  const uint32_t bg4 = bg * 0x01010101u;
  const int32_t delta = A.x0 - a.tx;                   // source column - destination column
  const int r16 = delta & 15, q = r16 >> 2, r = r16 & 3;
  // The class of a column changes only at the breakpoints (uniform per
  // sheet): five of the move, and the mask's two when one is folded in.
  // Vectors holding a breakpoint strictly inside, and the row's last
  // partial vector, are assembled byte by byte after the row's uniform
  // vectors -- one lane each, so the wave runs that path once per row.
  const int32_t bp[kMoveBp] = {a.tx, a.tx + aw, a.tx + sw, A.x0, A.x1 + 1,
                               kMask ? mk.x0 : 0, kMask ? mk.x1 + 1 : 0};
  // Deferred vectors (uniform): those holding a breakpoint strictly inside,
  // and the row's last partial vector, deduplicated.
  int32_t dvs[kMoveBp + 1];
  int nd = 0;
#pragma unroll
  for (int k = 0; k < kMoveBp + 1; k++) {
    const int32_t b = k < kMoveBp ? bp[k] : P.W;
    const bool has = k < kMoveBp ? (b > 0 && b < P.W && (b & 15)) : (P.W & 15) != 0;
    bool dup = false;
#pragma unroll
    for (int m = 0; m < kMoveBp + 1; m++)
      if (m < nd && dvs[m] == (b >> 4)) dup = true;
    if (has && !dup) dvs[nd++] = b >> 4;
  }
  // A column's class on a row is a function of four column facts (inside
  // the pasted columns, inside its copied part, inside the wiped area, inside
  // the mask) and four row facts; per row the sixteen column codes map to
  // classes (0 source, 1 background, 2 moved, 3 mask colour) through one
  // 32-bit table, so the column work is done once.
  auto col_code = [&](int32_t x) -> uint32_t {
    const int32_t u = x - a.tx;
    return (uint32_t)(u >= 0 && u < sw) | (uint32_t)(u < aw) << 1 |
           (uint32_t)(x >= A.x0 && x <= A.x1) << 2 | (uint32_t)(x >= mk.x0 && x <= mk.x1) << 3;
  };
  auto row_table = [&](int32_t y) -> uint32_t {
    const int32_t v = y - a.ty;
    const bool trow = v >= 0 && v < sh, mrow = trow && v < ah;
    const bool arow = y >= A.y0 && y <= A.y1;
    const bool krow = y >= mk.y0 && y <= mk.y1;
    uint32_t t = 0;
#pragma unroll
    for (int c = 0; c < 16; c++) {
      int cls = (trow && (c & 1)) ? ((mrow && (c & 2)) ? 2 : 1) : ((arow && (c & 4)) ? 1 : 0);
      if (kMask && cls == 0 && !(krow && (c & 8))) cls = 3;
      t |= (uint32_t)cls << (2 * c);
    }
    return t;
  };
  auto moved_row = [&](int32_t y) -> const uint8_t* {
    const int32_t v = y - a.ty;
    return sbase + (int64_t)(A.y0 + ((v >= 0 && v < ah) ? v : 0)) * P.pitch;
  };
  // kMoveVec vectors per lane per chunk of the row (192 slots: 155 used at A4 width)
  constexpr int kMoveVec = 3;
  for (int32_t vb = 0; vb < nv; vb += 64 * kMoveVec) {
    uint32_t cc[kMoveVec];   // column code, bit 4: no uniform vector here
    uint32_t reg[kMoveVec];  // counted columns (kRows)
#pragma unroll
    for (int k = 0; k < kMoveVec; k++) {
      const int32_t vi = vb + k * 64 + lane;
      const int32_t x0 = 16 * vi;
      bool deferred = vi >= nv || x0 + 16 > P.W;
#pragma unroll
      for (int j = 0; j < kMoveBp; j++) deferred |= bp[j] > x0 && bp[j] < x0 + 16;
      cc[k] = col_code(x0) | (deferred ? 16u : 0u);
      reg[k] = kRows ? cols16(x0, X.rx0, X.rx1) : 0u;
    }
#pragma unroll
    for (int ky = 0; ky < kMoveRows; ky++) {
      const int32_t y = y0 + ky;
      if (y >= y1) break;
      const uint8_t* srow = sbase + (int64_t)y * P.pitch;
      uint8_t* drow = dbase + (int64_t)y * P.pitch;
      const uint8_t* mrow_p = moved_row(y);
      const uint32_t tab = row_table(y);
      int cls[kMoveVec];
      uint4 lo[kMoveVec], hi[kMoveVec];
#pragma unroll
      for (int k = 0; k < kMoveVec; k++) {
        const int32_t x0 = 16 * (vb + k * 64 + lane);
        cls[k] = (cc[k] & 16u) ? -1 : (int)((tab >> (2 * (cc[k] & 15u))) & 3u);
        lo[k] = cls[k] == 3 ? make_uint4(mcol4, mcol4, mcol4, mcol4) : make_uint4(bg4, bg4, bg4, bg4);
        hi[k] = make_uint4(0, 0, 0, 0);
        if (cls[k] == 0) {
          lo[k] = *reinterpret_cast<const uint4*>(srow + x0);
        } else if (cls[k] == 2) {
          // a whole class-2 vector reads source columns inside [0, W), so
          // both aligned halves lie inside the (16-multiple) pitch
          const uint4* qp = reinterpret_cast<const uint4*>(mrow_p + ((x0 + delta) & ~15));
          lo[k] = qp[0];
          if (r16) hi[k] = qp[1];
        }
      }
#pragma unroll
      for (int k = 0; k < kMoveVec; k++) {
        const int32_t x0 = 16 * (vb + k * 64 + lane);
        if (cls[k] < 0) continue;
        uint4 out = lo[k];
        if (cls[k] == 2 && r16) {
          const uint32_t w[8] = {lo[k].x, lo[k].y, lo[k].z, lo[k].w,
                                 hi[k].x, hi[k].y, hi[k].z, hi[k].w};
          switch (q) {  // uniform over the sheet
            case 0: out = shift_bytes16<0>(w, r); break;
            case 1: out = shift_bytes16<1>(w, r); break;
            case 2: out = shift_bytes16<2>(w, r); break;
            default: out = shift_bytes16<3>(w, r); break;
          }
        }
        if (!kDry) *reinterpret_cast<uint4*>(drow + x0) = out;
        if (kRows && reg[k]) acc[ky] += dark16(out, reg[k], kadd);
      }
    }
  }
  // Deferred vectors: per byte, the class picks a byte of the source vector,
  // of the moved (realigned) vector, the background or the mask colour;
  // columns >= W stay 0.  The block's (row, deferred vector) pairs are
  // spread over all its lanes, one pair each (<= 8 x kMoveBlockRows <=
  // kThreads), so the byte work runs once per block rather than once per row
  // and wave.
  const int tid = threadIdx.x;
  const int32_t yr = yb + (nd ? tid / nd : 0);
  if (tid < nd * kMoveBlockRows && yr < yend) {
    const int di = tid - (tid / nd) * nd;
    int32_t vi = dvs[0];
#pragma unroll
    for (int m = 1; m < kMoveBp + 1; m++)
      if (m == di) vi = dvs[m];
    const int32_t x0 = 16 * vi;
    const int32_t y = yr;
    const uint8_t* srow = sbase + (int64_t)y * P.pitch;
    const uint8_t* mrow_p = moved_row(y);
    const uint32_t tab = row_table(y);
    // the aligned source halves of the moved bytes, each clamped into the row
    // (a clamped half only feeds bytes whose class is not 2)
    const int32_t al = (x0 + delta) & ~15;
    const int32_t alo = imin(imax(al, 0), (int32_t)P.pitch - 16);
    const int32_t ahi = imin(imax(al + 16, 0), (int32_t)P.pitch - 16);
    const uint4 sv = *reinterpret_cast<const uint4*>(srow + x0);
    const uint4 l = *reinterpret_cast<const uint4*>(mrow_p + alo);
    const uint4 h = *reinterpret_cast<const uint4*>(mrow_p + ahi);
    const uint32_t w[8] = {l.x, l.y, l.z, l.w, h.x, h.y, h.z, h.w};
    uint4 mv;
    switch (q) {
      case 0: mv = shift_bytes16<0>(w, r); break;
      case 1: mv = shift_bytes16<1>(w, r); break;
      case 2: mv = shift_bytes16<2>(w, r); break;
      default: mv = shift_bytes16<3>(w, r); break;
    }
    const uint32_t sw4[4] = {sv.x, sv.y, sv.z, sv.w};
    const uint32_t mw4[4] = {mv.x, mv.y, mv.z, mv.w};
    uint32_t o[4];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      uint32_t m0 = 0, m2 = 0, mb = 0, mc = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int32_t x = x0 + 4 * d + j;
        const uint32_t code = x < P.W ? col_code(x) : 16u;
        const uint32_t cls = (code & 16u) ? 4u : (tab >> (2 * code)) & 3u;
        const uint32_t byte = 0xFFu << (8 * j);
        m0 |= cls == 0 ? byte : 0u;
        m2 |= cls == 2 ? byte : 0u;
        mb |= cls == 1 ? byte : 0u;
        mc |= cls == 3 ? byte : 0u;
      }
      o[d] = (sw4[d] & m0) | (mw4[d] & m2) | (bg4 & mb) | (mcol4 & mc);
    }
    const uint4 ov = make_uint4(o[0], o[1], o[2], o[3]);
    if (!kDry) *reinterpret_cast<uint4*>(dbase + (int64_t)y * P.pitch + x0) = ov;
    if (kRows) {
      const uint32_t rg = cols16(x0, X.rx0, X.rx1);
      if (rg) atomicAdd(&rowcnt[y - yb], dark16(ov, rg, kadd));
    }
  }
  finish_rows();
}

void launch_move_rect(const PlaneRef& src, const PlaneRef& dst, const MoveArgs* args, int count,
                      hipStream_t st) {
  int gx = src.P.H < 1 ? 1 : (src.P.H > 1024 ? 1024 : src.P.H);
  if (src.P.fmt == F_GRAY8) {
    // kMoveRows consecutive rows per wave
    const int64_t blocks = (src.P.H + kMoveBlockRows - 1) / kMoveBlockRows;
    UPH_LAUNCH_DIAG(4, k_move_rect_g16<0>, dim3((unsigned)(blocks < 1 ? 1 : blocks), 1, count),
                    dim3(kThreads), 0, st, src, dst, args, MoveExtra{});
  } else if (src.P.fmt == F_Y400A) {
    hipLaunchKernelGGL(k_move_rect<F_Y400A>, dim3(gx, 1, count), dim3(kThreads), 0, st, src, dst,
                       args);
  } else {
    hipLaunchKernelGGL(k_move_rect_rgb, dim3(gx, 1, count), dim3(kThreads), 0, st, src, dst,
                       args);
  }
}

bool launch_move_rect_fused(const PlaneRef& src, const PlaneRef& dst, const MoveArgs* args,
                            const MoveExtra& x, int count, hipStream_t st) {
  if (src.P.fmt != F_GRAY8) return false;
  int64_t blocks = (src.P.H + kMoveBlockRows - 1) / kMoveBlockRows;
  if (x.ya1 > x.ya0 || x.yb1 > x.yb0) {  // row ranges (see k_move_rect_g16)
    if (!x.dry) return false;             // only a counting pass may skip rows
    blocks = (x.ya1 > x.ya0 ? (x.ya1 - x.ya0 + kMoveBlockRows - 1) / kMoveBlockRows : 0) +
             (x.yb1 > x.yb0 ? (x.yb1 - x.yb0 + kMoveBlockRows - 1) / kMoveBlockRows : 0);
    if (blocks == 0) return true;
  }
  const dim3 grid((unsigned)(blocks < 1 ? 1 : blocks), 1, count);
  const int mode = (x.masks ? 1 : 0) | (x.rows ? 2 : 0) | (x.dry ? 4 : 0);
  if (x.dry && x.masks) return false;
  switch (mode) {
    case 6: UPH_LAUNCH_DIAG(4, k_move_rect_g16<6>, grid, dim3(kThreads), 0, st, src, dst, args, x); break;
    case 1: UPH_LAUNCH_DIAG(4, k_move_rect_g16<1>, grid, dim3(kThreads), 0, st, src, dst, args, x); break;
    case 2: UPH_LAUNCH_DIAG(4, k_move_rect_g16<2>, grid, dim3(kThreads), 0, st, src, dst, args, x); break;
    case 3: UPH_LAUNCH_DIAG(4, k_move_rect_g16<3>, grid, dim3(kThreads), 0, st, src, dst, args, x); break;
    default: UPH_LAUNCH_DIAG(4, k_move_rect_g16<0>, grid, dim3(kThreads), 0, st, src, dst, args, x); break;
  }
  return true;
}

// ---------------------------------------------------------------------------
// center_mask, then apply_masks + align_mask (sheet_stages.c:415-499,
// masks.c:222-322) as ONE gather from the uncentred plane R, so that the
// centred plane C is never written: O(x, y) follows the align move's class
// rule back to C, C's centring rule back to R, and ends at a pixel of R or a
// constant (a background or the mask colour).  The classes are
// k_move_rect_g16's, stage by stage (move_class), so O is byte for byte what
// the two passes produce.  The border scan between the two moves reads only
// C's dark counts per row, which a dry centring pass (k_move_rect_g16 with
// kDry) counts from R without writing C.
//
// Columns: every stage's class changes only at a few columns (the move's
// five, the mask's two, and the first move's five seen through both possible
// outcomes of the second), so a row is a few intervals with one source
// offset or constant each.  A block (kMoveBlockRows rows of one sheet)
// finds the breakpoints, evaluates each (row, interval) once into LDS, and
// its lanes then write 16-byte vectors: one constant, or two aligned loads of
// R realigned by the interval's offset; vectors holding a breakpoint go byte
// by byte.
// ---------------------------------------------------------------------------
// k_move_rect_g16's class of (x, y) under move `a` (0 keep, 1 background,
// 2 moved: (x, y) become its source, 3 mask colour)
__device__ __forceinline__ int move_class(const MoveArgs& a, int32_t W, int32_t H, bool kmask,
                                          const Rect& mk, int32_t& x, int32_t& y) {
  const bool inmk = y >= mk.y0 && y <= mk.y1 && x >= mk.x0 && x <= mk.x1;
  if (!a.active) return kmask && !inmk ? 3 : 0;  // the identity: masked in place
  const Rect A = clip(a.area, W, H);
  const int32_t aw = A.x1 - A.x0 + 1, ah = A.y1 - A.y0 + 1;
  const int32_t sw = iabs(a.area.x0 - a.area.x1) + 1, sh = iabs(a.area.y0 - a.area.y1) + 1;
  const int32_t u = x - a.tx, v = y - a.ty;
  const bool trow = v >= 0 && v < sh, mrow = trow && v < ah;
  const bool arow = y >= A.y0 && y <= A.y1;
  const bool c1 = u >= 0 && u < sw, c2 = u < aw, c4 = x >= A.x0 && x <= A.x1;
  int cls = (trow && c1) ? ((mrow && c2) ? 2 : 1) : ((arow && c4) ? 1 : 0);
  if (kmask && cls == 0 && !inmk) cls = 3;
  if (cls == 2) {
    x = A.x0 + u;
    y = A.y0 + v;
  }
  return cls;
}

constexpr int kChainBp = 17;  // 7 of the align move and mask + 2 x 5 of the centring
#ifndef UPH_CHAIN_WAVES
#define UPH_CHAIN_WAVES 4
#endif
#ifndef UPH_CHAIN_OCC
#define UPH_CHAIN_OCC 1  // waves per SIMD the register budget must allow
#endif
constexpr int kChainThreads = 64 * UPH_CHAIN_WAVES;
constexpr int kChainRows = kMoveRows * UPH_CHAIN_WAVES;  // rows per block (kMoveRows a wave)
static_assert(kChainThreads >= kChainBp, "a thread per breakpoint");
struct ChainSheet {
  MoveArgs m1, m2;
  Rect mk;
  bool kmask;
  uint8_t mcol, bg1, bg2;
};
// The source of O(x, y): {-1, byte offset of the R pixel from (x, y)} or
// {constant, 0}
__device__ __forceinline__ int2 chain_cell(const ChainSheet& c, int32_t W, int32_t H,
                                           int64_t pitch, int32_t x, int32_t y) {
  int32_t sx = x, sy = y;
  const int c2 = move_class(c.m2, W, H, c.kmask, c.mk, sx, sy);
  if (c2 == 1) return make_int2(c.bg2, 0);
  if (c2 == 3) return make_int2(c.mcol, 0);
  const int c1 = move_class(c.m1, W, H, false, c.mk, sx, sy);
  if (c1 == 1) return make_int2(c.bg1, 0);
  return make_int2(-1, (int32_t)((int64_t)(sy - y) * pitch + (sx - x)));
}

__global__ void __launch_bounds__(kChainThreads, UPH_CHAIN_OCC) k_move_chain_g16(PlaneRef src, PlaneRef dst,
                                                             const MoveArgs* center,
                                                             const MaskArgs* masks,
                                                             const MoveArgs* align) {
  const int s = blockIdx.z;
  const Planes& P = src.P;
  const int32_t W = P.W, H = P.H;
  const int64_t pitch = P.pitch;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const int32_t yb = blockIdx.x * kChainRows;
  const int nrows = imin(kChainRows, H - yb);
  ChainSheet c;
  c.m1 = center[s];
  c.m2 = align[s];
  const MaskArgs& ma = masks[s];
  c.kmask = ma.n > 0;
  c.mk = c.kmask ? normalize(ma.m[0]) : Rect{INT_MIN / 2, INT_MIN / 2, INT_MAX / 2, INT_MAX / 2};
  c.mcol = gray_of(Px{ma.color[0], ma.color[1], ma.color[2]});
  c.bg1 = gray_of(Px{c.m1.bg[0], c.m1.bg[1], c.m1.bg[2]});
  c.bg2 = gray_of(Px{c.m2.bg[0], c.m2.bg[1], c.m2.bg[2]});
  __shared__ int32_t bp[kChainBp];
  __shared__ int32_t nbp_s, nd_s;
  __shared__ int32_t dv[kChainBp + 1];  // vectors holding a breakpoint (+ the row's partial one)
  __shared__ uint8_t live[kChainBp], imap[kChainBp + 1];
  __shared__ int2 cell[kChainRows][kChainBp + 1];
  __shared__ int32_t b[kChainBp];  // thread 0's candidate list (LDS, not scratch)
  if (threadIdx.x == 0) {
    // the columns where some stage's class can change (first column of the
    // new interval), sorted, unique, inside (0, W)
    int n = 0;
    auto add = [&](int32_t v) {
      if (v > 0 && v < W) b[n++] = v;
    };
    const MoveArgs& m2 = c.m2;
    int32_t d2 = 0;
    if (m2.active) {
      const Rect A = clip(m2.area, W, H);
      const int32_t sw = iabs(m2.area.x0 - m2.area.x1) + 1;
      add(m2.tx);
      add(m2.tx + (A.x1 - A.x0 + 1));
      add(m2.tx + sw);
      add(A.x0);
      add(A.x1 + 1);
      d2 = A.x0 - m2.tx;
    }
    if (c.kmask) {
      add(c.mk.x0);
      add(c.mk.x1 + 1);
    }
    if (c.m1.active) {
      const MoveArgs& m1 = c.m1;
      const Rect A = clip(m1.area, W, H);
      const int32_t sw = iabs(m1.area.x0 - m1.area.x1) + 1;
      const int32_t q[5] = {m1.tx, m1.tx + (A.x1 - A.x0 + 1), m1.tx + sw, A.x0, A.x1 + 1};
      for (int k = 0; k < 5; k++) {
        add(q[k]);                  // seen through a kept column of the align move
        if (m2.active) add(q[k] - d2);  // through a moved one
      }
    }
    for (int i = 1; i < n; i++)  // insertion sort
      for (int k = i; k > 0 && b[k - 1] > b[k]; k--) {
        const int32_t t = b[k];
        b[k] = b[k - 1];
        b[k - 1] = t;
      }
    int m = 0;
    for (int i = 0; i < n; i++)
      if (m == 0 || b[i] != bp[m - 1]) bp[m++] = b[i];
    nbp_s = m;
  }
  __syncthreads();
  int nbp = nbp_s;
  // every (row, interval) of the block: interval i starts at column 0 or bp[i-1]
  for (int t = threadIdx.x; t < nrows * (nbp + 1); t += blockDim.x) {
    const int r = t / (nbp + 1), i = t - r * (nbp + 1);
    cell[r][i] = chain_cell(c, W, H, pitch, i == 0 ? 0 : bp[i - 1], yb + r);
  }
  __syncthreads();
  // a breakpoint whose two intervals have the same source in every row of
  // the block changes nothing here: dropped (fewer byte-path vectors)
  if ((int)threadIdx.x < nbp) {
    const int k = threadIdx.x;
    bool same = true;
    for (int r = 0; r < nrows; r++) {
      const int2 a = cell[r][k], b = cell[r][k + 1];
      same = same && a.x == b.x && a.y == b.y;
    }
    live[k] = !same;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int m = 0;
    imap[0] = 0;
    for (int k = 0; k < nbp; k++)
      if (live[k]) {
        bp[m++] = bp[k];  // in place: m <= k
        imap[m] = (uint8_t)(k + 1);
      }
    nbp_s = m;
    int nd = 0;
    for (int k = 0; k < m; k++) {
      const int32_t v = bp[k] >> 4;
      if ((bp[k] & 15) && (nd == 0 || dv[nd - 1] != v)) dv[nd++] = v;
    }
    if ((W & 15) && (nd == 0 || dv[nd - 1] != (W >> 4))) dv[nd++] = W >> 4;
    nd_s = nd;
    for (int k = m; k < kChainBp; k++) bp[k] = INT_MAX;  // the register copy's padding
  }
  __syncthreads();
  nbp = nbp_s;
  int32_t bpr[kChainBp];  // the breakpoints in registers (INT_MAX past nbp)
#pragma unroll
  for (int k = 0; k < kChainBp; k++) bpr[k] = __builtin_amdgcn_readfirstlane(bp[k]);  // uniform: SGPRs
  auto interval = [&](int32_t x) {
    int i = 0;
#pragma unroll
    for (int k = 0; k < kChainBp; k++) i += bpr[k] <= x;
    return i;
  };
  const int lane = threadIdx.x & 63;
  const int32_t nv = (W + 15) >> 4;
  const int r0 = (threadIdx.x >> 6) * kMoveRows;  // the wave's rows of the block
  // uniform vectors: lanes along the row, the wave's kMoveRows rows
#ifndef UPH_CHAIN_KG
#define UPH_CHAIN_KG 4
#endif
  constexpr int kG = UPH_CHAIN_KG;  // rows whose loads are in flight together
  for (int32_t vi = lane; vi < nv; vi += 64) {
    const int32_t x0 = 16 * vi;
    const int il = interval(x0);
    if (x0 + 16 > W || il != interval(x0 + 15)) continue;  // byte path below
#pragma unroll
    for (int k0 = 0; k0 < kMoveRows; k0 += kG) {
      int2 ce[kG];
      int r16[kG];
      uint4 lo[kG], hi[kG];
#pragma unroll
      for (int j = 0; j < kG; j++) {
        // R bytes x0 + off .. + 15 of the row's cell: two aligned vectors
        // realigned by (off mod 16), the same for every vector of the interval
        const int r = r0 + k0 + j;
        ce[j] = r < nrows ? cell[r][imap[il]] : make_int2(0, 0);
        r16[j] = 0;
        lo[j] = hi[j] = make_uint4(0u, 0u, 0u, 0u);
        if (r < nrows && ce[j].x < 0) {
          const uint8_t* p = sbase + (int64_t)(yb + r) * pitch + x0 + ce[j].y;
          r16[j] = (int)((uintptr_t)p & 15u);
          const uint4* q = reinterpret_cast<const uint4*>(p - r16[j]);
          lo[j] = q[0];
          if (r16[j]) hi[j] = q[1];
        }
      }
#pragma unroll
      for (int j = 0; j < kG; j++) {
        const int r = r0 + k0 + j;
        if (r >= nrows) break;
        uint4 out;
        if (ce[j].x >= 0) {
          const uint32_t v4 = (uint32_t)ce[j].x * 0x01010101u;
          out = make_uint4(v4, v4, v4, v4);
        } else {
          const uint32_t w[8] = {lo[j].x, lo[j].y, lo[j].z, lo[j].w,
                                 hi[j].x, hi[j].y, hi[j].z, hi[j].w};
          const int ru = __builtin_amdgcn_readfirstlane(r16[j]);
          if (__builtin_amdgcn_ballot_w64(r16[j] != ru) == 0) {
            // the wave's vectors share one realignment (one cell, usually):
            // a uniform dword select, as k_move_rect_g16 does
            const int rb = ru & 3;
            switch (ru >> 2) {
              case 0: out = shift_bytes16<0>(w, rb); break;
              case 1: out = shift_bytes16<1>(w, rb); break;
              case 2: out = shift_bytes16<2>(w, rb); break;
              default: out = shift_bytes16<3>(w, rb); break;
            }
          } else {
            const int qd = r16[j] >> 2, rb = r16[j] & 3;
            uint32_t d[5];
#pragma unroll
            for (int m = 0; m < 5; m++)
              d[m] = qd == 0 ? w[m] : qd == 1 ? w[m + 1] : qd == 2 ? w[m + 2] : w[m + 3];
            out = make_uint4(__builtin_amdgcn_alignbyte(d[1], d[0], rb),
                             __builtin_amdgcn_alignbyte(d[2], d[1], rb),
                             __builtin_amdgcn_alignbyte(d[3], d[2], rb),
                             __builtin_amdgcn_alignbyte(d[4], d[3], rb));
          }
        }
        *reinterpret_cast<uint4*>(dbase + (int64_t)(yb + r) * pitch + x0) = out;
      }
    }
  }
  // vectors holding a breakpoint, and the row's partial last vector: a lane
  // per (row, vector), interval by interval, byte by byte; columns >= W are
  // written as 0
  const int nd = nd_s;
  for (int t = threadIdx.x; t < nrows * nd; t += blockDim.x) {
    const int r = t / nd, x0 = 16 * dv[t - r * nd];
    const int32_t y = yb + r;
    const uint8_t* srow = sbase + (int64_t)y * pitch;
    uint64_t o0 = 0, o1 = 0;
    const int il = interval(x0), ih = interval(imin(x0 + 15, W - 1));
    if (ih - il <= 3) {
      // the (at most three) breakpoints inside the vector; every byte's
      // source is independent of the others, so all 16 loads are in flight
      int32_t bk[3];
#pragma unroll
      for (int m = 0; m < 3; m++) bk[m] = il + m < ih ? bp[il + m] : INT_MAX;
      uint32_t v[16];
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int32_t x = x0 + j;
        const int i = il + (bk[0] <= x) + (bk[1] <= x) + (bk[2] <= x);
        const int2 ce = cell[r][imap[i]];
        v[j] = x >= W ? 0u : ce.x >= 0 ? (uint32_t)ce.x : (uint32_t)srow[x + ce.y];
      }
#pragma unroll
      for (int j = 0; j < 8; j++) {
        o0 |= (uint64_t)v[j] << (8 * j);
        o1 |= (uint64_t)v[8 + j] << (8 * j);
      }
    } else {
      for (int i = il; i <= ih; i++) {
        const int32_t s0 = imax(i == 0 ? 0 : bp[i - 1], x0);
        const int32_t s1 = imin(imin(i < nbp ? bp[i] : W, W), x0 + 16);
        const int2 ce = cell[r][imap[i]];
        for (int32_t x = s0; x < s1; x++) {
          const uint64_t v = ce.x >= 0 ? (uint64_t)ce.x : (uint64_t)srow[x + ce.y];
          const int j = x - x0;
          if (j < 8) o0 |= v << (8 * j);
          else o1 |= v << (8 * (j - 8));
        }
      }
    }
    *reinterpret_cast<uint4*>(dbase + (int64_t)y * pitch + x0) =
        make_uint4((uint32_t)o0, (uint32_t)(o0 >> 32), (uint32_t)o1, (uint32_t)(o1 >> 32));
  }
}

bool launch_move_chain(const PlaneRef& src, const PlaneRef& dst, const MoveArgs* center,
                       const MaskArgs* masks, const MoveArgs* align, int count, hipStream_t st) {
  if (src.P.fmt != F_GRAY8 || src.P.pitch * (int64_t)src.P.H >= (1ll << 31) || src.P.H < 1)
    return false;
  const int64_t blocks = (src.P.H + kChainRows - 1) / kChainRows;
  UPH_LAUNCH_DIAG(4, k_move_chain_g16, dim3((unsigned)blocks, 1, count), dim3(kChainThreads), 0, st,
                  src, dst, center, masks, align);
  return true;
}

// ---------------------------------------------------------------------------
// deskew_cpu + rotate (deskew.c:248-286) fused out of place: inside the mask
// rectangle (placed at mask.vertex[0], clipped to the image) the rotated
// pixel, elsewhere the source pixel.
//
// One workgroup per 64x16 output tile.  The source footprint of the tile's
// in-mask part (a rotated rectangle, plus the interpolation taps) is staged
// in LDS once -- white outside the image, which is what get_pixel returns --
// and every tap is then an LDS read.  The float expressions are untouched,
// so the result is identical to the direct gather, which remains the path
// for tiles whose footprint does not fit (rotations far beyond the default
// 5 degree range).
// ---------------------------------------------------------------------------
constexpr int kRotTW = 64, kRotTH = 16;
constexpr int kRotCap = 4096;  // staged pixels per tile

// LDS-staged window [x0, x0+w) x [y0, y0+h) of the source (channels: 1 for
// GRAY8/Y400A gray, 3 for RGB24); W/H are the image's, for the interpolators.
template <int FMT>
struct LdsSrc {
  const uint8_t* lds;
  int32_t x0, y0, w, h;
  int32_t W, H;
  Src<FMT> g;
  __device__ __forceinline__ Px at(int32_t x, int32_t y) const {
    const int32_t u = x - x0, v = y - y0;
    if (u < 0 || v < 0 || u >= w || v >= h) return g.at(x, y);  // never for in-bound tiles
    if (FMT == F_RGB24) {
      const uint8_t* q = lds + 3 * (v * w + u);
      return Px{q[0], q[1], q[2]};
    }
    const uint8_t q = lds[v * w + u];
    return Px{q, q, q};
  }
};

template <int FMT>
__global__ void __launch_bounds__(kThreads) k_rotate_mask(PlaneRef src, PlaneRef dst,
                                                          const RotateArgs* args, int interp) {
  constexpr int CH = FMT == F_RGB24 ? 3 : 1;
  __shared__ uint8_t stage[kRotCap * CH];
  const int s = blockIdx.z;
  const RotateArgs a = args[s];
  if (!a.active) return;
  const Planes& P = src.P;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const Rect nm = normalize(a.mask);
  const int32_t sw = nm.x1 - nm.x0 + 1, sh = nm.y1 - nm.y0 + 1;
  // center_of_rectangle (primitives.c:137-145)
  const float scx = nm.x0 + sw / 2.0f, scy = nm.y0 + sh / 2.0f;
  const float tcx = 0 + sw / 2.0f, tcy = 0 + sh / 2.0f;
  const Src<FMT> S{sbase, P.pitch, P.W, P.H};
  const int32_t tx0 = blockIdx.x * kRotTW, ty0 = blockIdx.y * kRotTH;
  // in-mask part of the tile, in mask coordinates (u, v)
  const int32_t u0 = imax(tx0, 0) - a.mask.x0, u1 = imin(tx0 + kRotTW, P.W) - 1 - a.mask.x0;
  const int32_t v0 = imax(ty0, 0) - a.mask.y0, v1 = imin(ty0 + kRotTH, P.H) - 1 - a.mask.y0;
  const int32_t cu0 = imax(u0, 0), cu1 = imin(u1, sw - 1);
  const int32_t cv0 = imax(v0, 0), cv1 = imin(v1, sh - 1);
  const bool any_in = cu0 <= cu1 && cv0 <= cv1;
  // source bounding box of the in-mask part (linear map: extremes at corners)
  int32_t bx0 = 0, by0 = 0, bw = 0, bh = 0;
  bool staged = false;
  if (any_in) {
    float mnx = 3.0e38f, mxx = -3.0e38f, mny = 3.0e38f, mxy = -3.0e38f;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int32_t u = c & 1 ? cu1 : cu0, v = c & 2 ? cv1 : cv0;
      const float X = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
      const float Y = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
      mnx = fminf(mnx, X);
      mxx = fmaxf(mxx, X);
      mny = fminf(mny, Y);
      mxy = fmaxf(mxy, Y);
    }
    // taps: cubic (int)c-1 .. (int)c+2 (trunc, so up to floor+3 for negative
    // c), bilinear floor..ceil, NN round; one more pixel each side absorbs
    // the rounding of per-pixel coordinates against the corner values
    bx0 = (int32_t)floorf(mnx) - 3;
    by0 = (int32_t)floorf(mny) - 3;
    bw = (int32_t)floorf(mxx) + 4 - bx0 + 1;
    bh = (int32_t)floorf(mxy) + 4 - by0 + 1;
    staged = bw > 0 && bh > 0 && (int64_t)bw * bh <= kRotCap;
  }
  if (staged) {
    // all loads of a round are issued before the LDS stores
    const int n = bw * bh;
    for (int base = 0; base < n; base += 8 * kThreads) {
      uint8_t v[8][CH];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = base + k * kThreads + threadIdx.x;
        const int32_t x = bx0 + i % bw, y = by0 + i / bw;
#pragma unroll
        for (int c = 0; c < CH; c++) v[k][c] = 255;
        if (i < n && x >= 0 && y >= 0 && x < P.W && y < P.H) {
          const Px p = load_px_row<FMT>(sbase + (int64_t)y * P.pitch, x);
          v[k][0] = p.r;
          if (CH == 3) {
            v[k][1] = p.g;
            v[k][2] = p.b;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = base + k * kThreads + threadIdx.x;
        if (i < n) {
#pragma unroll
          for (int c = 0; c < CH; c++) stage[i * CH + c] = v[k][c];
        }
      }
    }
  }
  __syncthreads();
  const LdsSrc<FMT> L{stage, bx0, by0, bw, bh, P.W, P.H, S};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t x = tx0 + lane;
  if (x >= P.W) return;
  const int32_t u = x - a.mask.x0;
#pragma unroll
  for (int k = 0; k < kRotTH / 4; k++) {
    const int32_t y = ty0 + w + 4 * k;
    if (y >= P.H) break;
    uint8_t* drow = dbase + (int64_t)y * P.pitch;
    const int32_t v = y - a.mask.y0;
    if (u >= 0 && u < sw && v >= 0 && v < sh) {
      const float srcX = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
      const float srcY = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
      if (FMT != F_RGB24 && staged && interp == UPHIP_INTERP_CUBIC) {
        // gray bicubic straight from the window: the 4x4 taps of (int)srcX,
        // (int)srcY lie inside it by construction of the bounding box
        const int ix = (int)srcX, iy = (int)srcY;
        const uint8_t* t = stage + (iy - 1 - by0) * bw + (ix - 1 - bx0);
        const float fx = srcX - ix;
        uint8_t col[4];
#pragma unroll
        for (int r = 0; r < 4; r++, t += bw) col[r] = cubic_scale(fx, t[0], t[1], t[2], t[3]);
        const uint8_t o = cubic_scale(srcY - iy, col[0], col[1], col[2], col[3]);
        store_px_row<FMT>(drow, x, Px{o, o, o});
        continue;
      }
      const Px o = staged ? interpolate<FMT>(L, srcX, srcY, interp)
                          : interpolate<FMT>(S, srcX, srcY, interp);
      store_px_row<FMT>(drow, x, o);
    } else {
      copy_px_raw<FMT>(drow, x, sbase + (int64_t)y * P.pitch, x);
    }
  }
}

// cubic_scale (interpolate.c:24-31) on integer taps.  Its integer-valued
// subexpressions -- 2a-5b+4c-d, 3(b-c)+d-a and c-a -- are exact in float
// (|x| < 2^24), so they are formed in int and converted; the six rounding
// operations remain, in the reference's order:
//   b + (0.5f*f) * ((c-a) + f * ((2a-5b+4c-d) + f * (3(b-c)+d-a)))
__device__ __forceinline__ uint8_t cubic_int(float f, float h, int a, int b, int c, int d) {
  const float s2 = (float)(3 * (b - c) + d - a);
  const float s1 = (float)(2 * a - 5 * b + 4 * c - d);
  const float u = s1 + f * s2;
  const float v = (float)(c - a) + f * u;
  const int r = (int)((float)b + h * v);
  return (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));  // av_clip_uint8
}

// deskew rotate for a gray plane with bicubic interpolation (Y400A):
// k_rotate_mask's tiling and staging, with the taps read straight from the
// window and no other interpolation code in the kernel.
constexpr int kRotGH = 32;     // output rows per tile of the gray bicubic kernel
constexpr int kRotGCap = 6144; // its staged pixels per tile

template <int FMT>
__global__ void __launch_bounds__(kThreads) k_rotate_cubic_gray(PlaneRef src, PlaneRef dst,
                                                                const RotateArgs* args) {
  __shared__ uint32_t stage32[kRotGCap / 4];
  uint8_t* stage = reinterpret_cast<uint8_t*>(stage32);
  // XCD-aware tile order: neighbouring windows share rows, fetched into one L2
  int txi, tyi, s;
  xcd_block(&txi, &tyi, &s);
  const RotateArgs a = args[s];
  if (!a.active) return;
  const Planes& P = src.P;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const Rect nm = normalize(a.mask);
  const int32_t sw = nm.x1 - nm.x0 + 1, sh = nm.y1 - nm.y0 + 1;
  const float scx = nm.x0 + sw / 2.0f, scy = nm.y0 + sh / 2.0f;  // primitives.c:137-145
  const float tcx = 0 + sw / 2.0f, tcy = 0 + sh / 2.0f;
  const int32_t tx0 = txi * kRotTW, ty0 = tyi * kRotGH;
  const int32_t u0 = imax(tx0, 0) - a.mask.x0, u1 = imin(tx0 + kRotTW, P.W) - 1 - a.mask.x0;
  const int32_t v0 = imax(ty0, 0) - a.mask.y0, v1 = imin(ty0 + kRotGH, P.H) - 1 - a.mask.y0;
  const int32_t cu0 = imax(u0, 0), cu1 = imin(u1, sw - 1);
  const int32_t cv0 = imax(v0, 0), cv1 = imin(v1, sh - 1);
  int32_t bx0 = 0, by0 = 0, bw = 0, bh = 0;
  bool staged = false;
  if (cu0 <= cu1 && cv0 <= cv1) {
    float mnx = 3.0e38f, mxx = -3.0e38f, mny = 3.0e38f, mxy = -3.0e38f;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int32_t u = c & 1 ? cu1 : cu0, v = c & 2 ? cv1 : cv0;
      const float X = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
      const float Y = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
      mnx = fminf(mnx, X);
      mxx = fmaxf(mxx, X);
      mny = fminf(mny, Y);
      mxy = fmaxf(mxy, Y);
    }
    bx0 = (int32_t)floorf(mnx) - 3;
    by0 = (int32_t)floorf(mny) - 3;
    bw = (int32_t)floorf(mxx) + 4 - bx0 + 1;
    bh = (int32_t)floorf(mxy) + 4 - by0 + 1;
    staged = bw > 0 && bh > 0;
  }
  // gray planes stage whole aligned dwords: row r of the window starts at
  // byte `lead` of a `sstride`-byte LDS row
  const int32_t xa = bx0 >= 0 ? (bx0 & ~3) : -((-bx0 + 3) & ~3);
  const int lead = FMT == F_GRAY8 ? bx0 - xa : 0;
  const int nd = (lead + bw + 3) >> 2;
  const int sstride = FMT == F_GRAY8 ? 4 * nd : bw;
  staged = staged && (int64_t)sstride * bh <= kRotGCap;
  if (staged && FMT == F_GRAY8) {
    const int n = nd * bh;
    for (int b0 = 0; b0 < n; b0 += 8 * kThreads) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = b0 + k * kThreads + threadIdx.x;
        const int r = i / nd;
        const int32_t xd = xa + 4 * (i - r * nd), y = by0 + r;
        const bool row_ok = (y >= 0) & (y < P.H);
        const uint8_t* row = sbase + (int64_t)imin(imax(y, 0), P.H - 1) * P.pitch;
        // interior dwords: one aligned load (xd is a multiple of 4)
        v[k] = *reinterpret_cast<const uint32_t*>(row + imin(imax(xd, 0), (int32_t)P.pitch - 4));
        if (!row_ok) v[k] = 0xFFFFFFFFu;
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = b0 + k * kThreads + threadIdx.x;
        if (i >= n) continue;
        const int r = i / nd;
        const int32_t xd = xa + 4 * (i - r * nd), y = by0 + r;
        uint32_t w4 = v[k];
        if ((y >= 0) & (y < P.H) & ((xd < 0) | (xd + 3 >= P.W))) {
          // a dword across the image edge: white outside, bytes inside
          const uint8_t* row = sbase + (int64_t)y * P.pitch;
          w4 = 0;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int32_t x = xd + j;
            const uint32_t b = (x >= 0 && x < P.W) ? row[x] : 255u;
            w4 |= b << (8 * j);
          }
        }
        stage32[i] = w4;
      }
    }
  } else if (staged) {
    // unconditional clamped loads (white off the image), all of a round in flight
    const int n = bw * bh;
    for (int b0 = 0; b0 < n; b0 += 8 * kThreads) {
      uint8_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = b0 + k * kThreads + threadIdx.x;
        const int r = i / bw;
        const int32_t x = bx0 + (i - r * bw), y = by0 + r;
        const bool ok = (x >= 0) & (y >= 0) & (x < P.W) & (y < P.H);
        const uint8_t q = load_px_row<FMT>(sbase + (int64_t)imin(imax(y, 0), P.H - 1) * P.pitch,
                                           imin(imax(x, 0), P.W - 1)).r;
        v[k] = ok ? q : (uint8_t)255;
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = b0 + k * kThreads + threadIdx.x;
        if (i < n) stage[i] = v[k];
      }
    }
  }
  __syncthreads();
  const Src<FMT> S{sbase, P.pitch, P.W, P.H};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t x = tx0 + lane;
  if (x >= P.W) return;
  const int32_t u = x - a.mask.x0;
#pragma unroll
  for (int k = 0; k < kRotGH / 4; k++) {
    const int32_t y = ty0 + w + 4 * k;
    if (y >= P.H) break;
    uint8_t* drow = dbase + (int64_t)y * P.pitch;
    const int32_t v = y - a.mask.y0;
    if (u >= 0 && u < sw && v >= 0 && v < sh) {
      const float srcX = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
      const float srcY = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
      uint8_t o;
      if (staged) {
        const int ix = (int)srcX, iy = (int)srcY;  // interp_bicubic truncates
        const float fx = srcX - ix, fy = srcY - iy;
        const float hx = 0.5f * fx, hy = 0.5f * fy;
        const uint8_t* t = stage + (iy - 1 - by0) * sstride + lead + (ix - 1 - bx0);
        int col[4];
#pragma unroll
        for (int r = 0; r < 4; r++, t += sstride)
          col[r] = cubic_int(fx, hx, t[0], t[1], t[2], t[3]);
        o = cubic_int(fy, hy, col[0], col[1], col[2], col[3]);
      } else {
        o = interp_bicubic(S, srcX, srcY).r;
      }
      store_px_row<FMT>(drow, x, Px{o, o, o});
    } else {
      copy_px_raw<FMT>(drow, x, sbase + (int64_t)y * P.pitch, x);
    }
  }
}

// ---------------------------------------------------------------------------
// deskew rotate, GRAY8 + bicubic (the default pipeline): 256 x 32 output tiles,
// four horizontally adjacent pixels per lane and row, so one dword store per
// lane and the float work in pairs of pixels on packed FP32 (v_pk_mul/add/fma).
//   * the window is staged with a fixed 288-byte row stride, so the four tap
//     rows of a pixel are one ds_read2_b32 each at immediate offsets, and
//     v_alignbyte extracts its four taps;
//   * the integer-valued terms of cubic_scale (2a-5b+4c-d, 3(b-c)+d-a, c-a)
//     are formed by exact packed FMAs on float-valued bytes (every
//     intermediate is an integer below 2^24); the six rounding operations stay
//     separate multiplies and adds in the reference's order
//     (interpolate.c:24-31), so results are bit-identical.
// ---------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kRQW = 256;              // output columns per tile (4 per lane)
constexpr int kRQH = 32;               // output rows per tile
constexpr int kRQStride = 72;          // staged row stride in dwords (>= window 269 B)
constexpr int kRQRows = 84;            // staged rows
constexpr int kRQWords = kRQStride * kRQRows + 2;

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat2(float v) { return f2{v, v}; }

// cubic_scale on float-valued taps, truncated and clipped like av_clip_uint8
// (the result is an integer-valued float).  The integer-valued terms are
// formed from the differences ba = b-a, ca = c-a, da = d-a:
//   2a-5b+4c-d = -5ba + 4ca - da,   3(b-c)+d-a = 3(ba-ca) + da
// The integer coefficients of cubic_scale (interpolate.c:24-31) for taps
// a..d, exact in fp32 (|values| <= 1530), in six packed operations:
//   ca = c - a,  s2 = 3(b - c) + (d - a),  s1 = 2a - 5b + 4c - d
//                                         = -5(b - c) - ((d - a) + (c - a))
__device__ __forceinline__ void cubic_terms(f2 a, f2 b, f2 c, f2 d, f2& ca, f2& s1, f2& s2) {
  const f2 e = d - a, g = b - c;
  ca = c - a;
  s2 = fma2(splat2(3.0f), g, e);
  s1 = fma2(splat2(-5.0f), g, -(e + ca));
}

__device__ __forceinline__ f2 cubic2(f2 f, f2 h, f2 a, f2 b, f2 c, f2 d) {
  f2 ca, s1, s2;
  cubic_terms(a, b, c, d, ca, s1, s2);  // exact
  const f2 u = s1 + f * s2;
  const f2 v = ca + f * u;
  const f2 r = b + h * v;
  return f2{__builtin_amdgcn_fmed3f(__builtin_truncf(r.x), 0.0f, 255.0f),
            __builtin_amdgcn_fmed3f(__builtin_truncf(r.y), 0.0f, 255.0f)};
}

// byte K of w as a float.  Inline asm keeps the value opaque: otherwise the
// compiler turns differences of converted bytes back into integer subtracts
// plus conversions, which defeats the packed arithmetic.
template <int K>
__device__ __forceinline__ float ubyte_f(uint32_t w) {
  float r;
  if constexpr (K == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(w));
  else if constexpr (K == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(w));
  else if constexpr (K == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(w));
  else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(w));
  return r;
}
template <int K>
__device__ __forceinline__ f2 tap2(uint32_t p, uint32_t q) {
  return f2{ubyte_f<K>(p), ubyte_f<K>(q)};
}

__global__ void __launch_bounds__(kThreads) k_rotate_cubic_g8(PlaneRef src, PlaneRef dst,
                                                              const RotateArgs* args) {
  __shared__ uint32_t win[kRQWords];
  int txi, tyi, s;
  xcd_block(&txi, &tyi, &s);  // neighbouring windows share rows, fetched into one L2
  const RotateArgs a = args[s];
  if (!a.active) return;
  const Planes& P = src.P;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const Rect nm = normalize(a.mask);
  const int32_t sw = nm.x1 - nm.x0 + 1, sh = nm.y1 - nm.y0 + 1;
  const float scx = nm.x0 + sw / 2.0f, scy = nm.y0 + sh / 2.0f;  // primitives.c:137-145
  const float tcx = 0 + sw / 2.0f, tcy = 0 + sh / 2.0f;
  const int32_t tx0 = txi * kRQW, ty0 = tyi * kRQH;
  const int32_t u0 = imax(tx0, 0) - a.mask.x0, u1 = imin(tx0 + kRQW, P.W) - 1 - a.mask.x0;
  const int32_t v0 = imax(ty0, 0) - a.mask.y0, v1 = imin(ty0 + kRQH, P.H) - 1 - a.mask.y0;
  const int32_t cu0 = imax(u0, 0), cu1 = imin(u1, sw - 1);
  const int32_t cv0 = imax(v0, 0), cv1 = imin(v1, sh - 1);
  // source window of the tile's in-mask pixels (their 4x4 taps included)
  int32_t bx0 = 0, by0 = 0, bw = 0, bh = 0;
  if (cu0 <= cu1 && cv0 <= cv1) {
    float mnx = 3.0e38f, mxx = -3.0e38f, mny = 3.0e38f, mxy = -3.0e38f;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int32_t u = c & 1 ? cu1 : cu0, v = c & 2 ? cv1 : cv0;
      const float X = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
      const float Y = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
      mnx = fminf(mnx, X);
      mxx = fmaxf(mxx, X);
      mny = fminf(mny, Y);
      mxy = fmaxf(mxy, Y);
    }
    bx0 = (int32_t)floorf(mnx) - 3;
    by0 = (int32_t)floorf(mny) - 3;
    bw = (int32_t)floorf(mxx) + 4 - bx0 + 1;
    bh = (int32_t)floorf(mxy) + 4 - by0 + 1;
  }
  const int32_t xa = bx0 >= 0 ? (bx0 & ~3) : -((-bx0 + 3) & ~3);  // window start, dword aligned
  const int lead = bx0 - xa;
  const int nd = (lead + bw + 3) >> 2;                               // dwords per window row
  const bool staged = bw > 0 && bh > 0 && nd < kRQStride && bh <= kRQRows;
  if (staged) {
    // row of flat dword index i: i / nd as a multiply-high (exact for
    // i * (m*nd - 2^32) < 2^32, far beyond these sizes)
    const uint32_t m = nd > 1 ? (uint32_t)((0xFFFFFFFFull / (uint32_t)nd) + 1) : 0u;
    const int n = nd * bh;
    for (int b0 = 0; b0 < n; b0 += 8 * kThreads) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = b0 + k * kThreads + threadIdx.x;
        const int r = nd > 1 ? (int)__umulhi((uint32_t)i, m) : i;
        const int32_t xd = xa + 4 * (i - r * nd), y = by0 + r;
        const uint8_t* row = sbase + (int64_t)imin(imax(y, 0), P.H - 1) * P.pitch;
        v[k] = *reinterpret_cast<const uint32_t*>(row + imin(imax(xd, 0), (int32_t)P.pitch - 4));
        if ((y < 0) | (y >= P.H)) v[k] = 0xFFFFFFFFu;
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = b0 + k * kThreads + threadIdx.x;
        if (i >= n) continue;
        const int r = nd > 1 ? (int)__umulhi((uint32_t)i, m) : i;
        const int j = i - r * nd;
        const int32_t xd = xa + 4 * j, y = by0 + r;
        uint32_t w4 = v[k];
        if ((y >= 0) & (y < P.H) & ((xd < 0) | (xd + 3 >= P.W))) {
          // a dword across the image edge: white outside, bytes inside
          const uint8_t* row = sbase + (int64_t)y * P.pitch;
          w4 = 0;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int32_t x = xd + q;
            const uint32_t b = (x >= 0 && x < P.W) ? row[x] : 255u;
            w4 |= b << (8 * q);
          }
        }
        win[r * kRQStride + j] = w4;
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t xl = tx0 + 4 * lane;
  if (xl >= P.W) return;
  // per-lane terms of the source coordinates (constant down the column):
  //   srcX = (scx + (u - tcx) cos) + (v - tcy) sin
  //   srcY = (scy + (v - tcy) cos) - (u - tcx) sin
  float ax[4], bs[4];
  bool colin[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int32_t u = xl + j - a.mask.x0;
    const float cu = u - tcx;
    ax[j] = scx + cu * a.cosval;
    bs[j] = cu * a.sinval;
    colin[j] = (u >= 0) & (u < sw) & (xl + j < P.W);
  }
  const f2 AX0{ax[0], ax[1]}, AX1{ax[2], ax[3]}, BS0{bs[0], bs[1]}, BS1{bs[2], bs[3]};
  const int base_off = (-1 - by0) * (4 * kRQStride) + lead - 1 - bx0;  // tap (ix-1, iy-1)
  const Src<F_GRAY8> S{sbase, P.pitch, P.W, P.H};
#pragma unroll 2
  for (int k = 0; k < kRQH / 4; k++) {
    const int32_t y = ty0 + w + 4 * k;
    if (y >= P.H) break;
    const int32_t v = y - a.mask.y0;
    const bool rowin = (v >= 0) & (v < sh);
    const float cv = v - tcy;
    const f2 VS = splat2(cv * a.sinval), VC = splat2(scy + cv * a.cosval);
    const f2 SX[2] = {AX0 + VS, AX1 + VS};
    const f2 SY[2] = {VC - BS0, VC - BS1};
    const uint8_t* srow = sbase + (int64_t)y * P.pitch;
    uint32_t out = 0;
    if (staged) {
#pragma unroll
      for (int pr = 0; pr < 2; pr++) {
        const int ix0 = (int)SX[pr].x, ix1 = (int)SX[pr].y;  // interp_bicubic truncates
        const int iy0 = (int)SY[pr].x, iy1 = (int)SY[pr].y;
        const f2 fx = SX[pr] - f2{(float)ix0, (float)ix1};
        const f2 fy = SY[pr] - f2{(float)iy0, (float)iy1};
        const f2 hx = 0.5f * fx, hy = 0.5f * fy;
        const bool in0 = rowin & colin[2 * pr], in1 = rowin & colin[2 * pr + 1];
        const int o0 = in0 ? base_off + iy0 * (4 * kRQStride) + ix0 : 0;
        const int o1 = in1 ? base_off + iy1 * (4 * kRQStride) + ix1 : 0;
        const uint32_t* w0 = win + (o0 >> 2);
        const uint32_t* w1 = win + (o1 >> 2);
        f2 col[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const uint32_t p = __builtin_amdgcn_alignbyte(w0[r * kRQStride + 1], w0[r * kRQStride], o0);
          const uint32_t q = __builtin_amdgcn_alignbyte(w1[r * kRQStride + 1], w1[r * kRQStride], o1);
          col[r] = cubic2(fx, hx, tap2<0>(p, q), tap2<1>(p, q), tap2<2>(p, q), tap2<3>(p, q));
        }
        const f2 o = cubic2(fy, hy, col[0], col[1], col[2], col[3]);
        // integer-valued in [0, 255]: the conversion is exact whatever its rounding
        out = __builtin_amdgcn_cvt_pk_u8_f32(o.x, 2 * pr, out);
        out = __builtin_amdgcn_cvt_pk_u8_f32(o.y, 2 * pr + 1, out);
      }
    } else {
      // window too tall for LDS (large angles): taps from the frame
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const f2 sx = SX[j >> 1], sy = SY[j >> 1];
        const float fx = (j & 1) ? sx.y : sx.x, fy = (j & 1) ? sy.y : sy.x;
        if (rowin & colin[j]) out |= (uint32_t)interp_bicubic(S, fx, fy).r << (8 * j);
      }
    }
    // outside the mask the pixel is copied unchanged (deskew.c:268-286)
    uint32_t inmask = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) inmask |= (rowin & colin[j]) ? 0xFFu << (8 * j) : 0u;
    uint8_t* drow = dbase + (int64_t)y * P.pitch;
    if (xl + 3 < P.W) {
      if (inmask != 0xFFFFFFFFu)
        out = (out & inmask) | (*reinterpret_cast<const uint32_t*>(srow + xl) & ~inmask);
      *reinterpret_cast<uint32_t*>(drow + xl) = out;
    } else {
      for (int j = 0; xl + j < P.W; j++)
        drow[xl + j] = (inmask >> (8 * j)) & 1 ? (uint8_t)(out >> (8 * j)) : srow[xl + j];
    }
  }
}

// ---------------------------------------------------------------------------
// deskew rotate, GRAY8 + bicubic, float window (the default pipeline's
// dominant kernel).  128 x 48 output tiles; the tile's source window is
// staged once as fp32 (one conversion per staged byte instead of one per
// tap), so the taps of a pixel come straight out of LDS in the pairs the
// packed FP32 ops consume:
//   * a lane owns output columns tx0+lane and tx0+64+lane (A, B); the row
//     cubics of one pixel run two tap rows at a time, each tap pair (row r,
//     row r+1) one ds_read2_b32 at offsets (k, kRFS+k);
//   * the vertical cubic runs A and B as one packed pair;
//   * lanes read consecutive columns (a wave whose pixels straddle a row
//     boundary meets at most two-way bank conflicts);
//   * all-white stretches of a tile row (the page background) are detected
//     from per-row non-white masks built while staging and skip the math;
//   * each wave buffers its six output rows in LDS and stores them 8 bytes
//     per lane at the end (no global load after a store).
// Every rounding operation of cubic_scale (interpolate.c:24-31) stays a
// separate multiply or add in the reference's order, as in cubic2.
// ---------------------------------------------------------------------------
constexpr int kRFW = 128;   // output columns per tile (2 per lane)
#ifndef UPH_ROT_TALL
#define UPH_ROT_TALL 0
#endif
constexpr int kRFH = UPH_ROT_TALL ? 96 : 48;  // output rows per tile (6 or 12 per wave)
constexpr int kRFS = 144;   // staged row stride in floats (>= 141-float window rows at 5 deg)
constexpr int kRFT = 512;   // threads per tile: 8 waves, kRFH / 8 consecutive rows each
constexpr int kRFWaves = kRFT / 64;

// The 16 taps of pixels A and B as row pairs: t[p][j] = {tap row 2q, tap row
// 2q+1} of column j for p = 2*pixel + q.  a[p] is the LDS byte address of
// (column 0, row 2q).  One ds_read2_b32 per pair (offsets k and kRFS + k,
// which the compiler would instead merge as k, k+1 and then shuffle), all 16
// in flight before the one wait.
#define UPH_TAP_PAIR(o, b, k) \
  "ds_read2_b32 %" #o ", %" #b " offset0:" #k " offset1:" UPH_STR(UPH_ROWOFF_##k) "\n\t"
#define UPH_STR2(x) #x
#define UPH_STR(x) UPH_STR2(x)
#define UPH_ROWOFF_0 144
#define UPH_ROWOFF_1 145
#define UPH_ROWOFF_2 146
#define UPH_ROWOFF_3 147
static_assert(kRFS == 144, "tap pair offsets are spelled out for a 144-float row stride");
// Issued in pair order t[0], t[1] (pixel A), t[2], t[3] (pixel B) with no
// wait: the caller waits for A's eight (lds_wait_a) and computes A's row
// cubics while B's are still in flight (LDS returns in order).
__device__ __forceinline__ void lds_taps16(const uint32_t (&a)[4], f2 (&t)[4][4]) {
  asm volatile(UPH_TAP_PAIR(0, 16, 0) UPH_TAP_PAIR(1, 16, 1) UPH_TAP_PAIR(2, 16, 2)
               UPH_TAP_PAIR(3, 16, 3) UPH_TAP_PAIR(4, 17, 0) UPH_TAP_PAIR(5, 17, 1)
               UPH_TAP_PAIR(6, 17, 2) UPH_TAP_PAIR(7, 17, 3) UPH_TAP_PAIR(8, 18, 0)
               UPH_TAP_PAIR(9, 18, 1) UPH_TAP_PAIR(10, 18, 2) UPH_TAP_PAIR(11, 18, 3)
               UPH_TAP_PAIR(12, 19, 0) UPH_TAP_PAIR(13, 19, 1) UPH_TAP_PAIR(14, 19, 2)
               UPH_TAP_PAIR(15, 19, 3)
               : "=&v"(t[0][0]), "=&v"(t[0][1]), "=&v"(t[0][2]), "=&v"(t[0][3]),
                 "=&v"(t[1][0]), "=&v"(t[1][1]), "=&v"(t[1][2]), "=&v"(t[1][3]),
                 "=&v"(t[2][0]), "=&v"(t[2][1]), "=&v"(t[2][2]), "=&v"(t[2][3]),
                 "=&v"(t[3][0]), "=&v"(t[3][1]), "=&v"(t[3][2]), "=&v"(t[3][3])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
               : "memory");
}
// Wait until <= N LDS operations are outstanding; the taps of pairs p0, p0+1
// become defined here (no use of them can be scheduled above the wait).
template <int N>
__device__ __forceinline__ void lds_wait_pairs(f2 (&u)[4], f2 (&v)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(v[0]), "+v"(v[1]),
                 "+v"(v[2]), "+v"(v[3])
               : "n"(N)
               : "memory");
}

// Wait until <= N LDS operations are outstanding: tap pair t becomes
// defined here; `prev` (the previous pair's result) must be computed above
// the wait, so each pair's arithmetic overlaps the later pairs' reads.
template <int N>
__device__ __forceinline__ void lds_wait_pair(f2 (&t)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)"
               : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3])
               : "n"(N)
               : "memory");
}
template <int N>
__device__ __forceinline__ void lds_wait_pair_after(f2 (&t)[4], f2& prev) {
  asm volatile("s_waitcnt lgkmcnt(%5)"
               : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(prev)
               : "n"(N)
               : "memory");
}

// one packed row cubic (rows 2q, 2q+1 of one pixel), clamped like cubic_scale
__device__ __forceinline__ f2 cubic2_row_u(f2 f, f2 h, const f2 (&t)[4]) {
  f2 ca, s1, s2;
  cubic_terms(t[0], t[1], t[2], t[3], ca, s1, s2);  // exact
  f2 u = f * s2;
  u = s1 + u;
  u = f * u;
  u = ca + u;
  u = h * u;
  return t[1] + u;
}
// cubic2_row_u on two independent pairs step by step, so the dependent
// packed operations of one chain fill the other's wait states
__device__ __forceinline__ void cubic2_row_u2(f2 f0, f2 h0, const f2 (&t0)[4], f2 f1, f2 h1,
                                              const f2 (&t1)[4], f2& o0, f2& o1) {
  f2 ca0, s10, s20, ca1, s11, s21;
  cubic_terms(t0[0], t0[1], t0[2], t0[3], ca0, s10, s20);
  cubic_terms(t1[0], t1[1], t1[2], t1[3], ca1, s11, s21);
  f2 u0 = f0 * s20, u1 = f1 * s21;
  u0 = s10 + u0;
  u1 = s11 + u1;
  u0 = f0 * u0;
  u1 = f1 * u1;
  u0 = ca0 + u0;
  u1 = ca1 + u1;
  u0 = h0 * u0;
  u1 = h1 * u1;
  o0 = t0[1] + u0;
  o1 = t1[1] + u1;
}
// cubic_scale's truncation and clamp of one result
__device__ __forceinline__ float clamp_t255(float u) {
  return __builtin_amdgcn_fmed3f(__builtin_truncf(u), 0.0f, 255.0f);
}

// v from the lane given by the quad permutation CTRL (DPP quad_perm)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Byte offset of row y (0 <= y < H) as a 32-bit product: the launcher only
// picks k_rotate_cubic_g8f when pitch * H < 2^31 (one scalar multiply per row
// instead of a 64-bit product).
__device__ __forceinline__ uint32_t row_off(int32_t y, int64_t pitch) {
  return (uint32_t)y * (uint32_t)pitch;
}

#ifndef UPH_ROT_MINB
#define UPH_ROT_MINB 8
#endif
// 1: one block barrier per in-mask tile (staging): every wave finds the
// window bounds itself, and the column sums are flushed by the last wave to
// finish (an LDS arrival counter) instead of after a second barrier.  Measured
// slower (1.11 vs 1.08 ms a 64-sheet launch: the corners' VALU in every wave
// costs more than the barriers), kept off.
#ifndef UPH_ROT_V2
#define UPH_ROT_V2 0
#endif
#ifndef UPH_ROT_FULL
#define UPH_ROT_FULL 1  // the branch-free row loop for full tiles
#endif
#ifndef UPH_ROT_EARLY
#define UPH_ROT_EARLY 1  // 0: the column-sum zero barrier in every tile (round-4 form)
#endif
#ifndef UPH_ROT_PAIRS
// 1: a pixel's two row pairs interleaved after one wait (fewer wait states,
// less overlap with the tap reads: A/B 0.99 vs 0.975 ms a launch, kept off)
#define UPH_ROT_PAIRS 0
#endif
#ifndef UPH_ROT_UNIFORM
#define UPH_ROT_UNIFORM 0  // 1: skip wave rows of uniform 4x4 windows (A/B: see DESIGN §5)
#endif
#ifdef UPHIP_DIAG
// tuning build: per-phase shader clocks of wave 0 of every in-mask tile
// (UPHIP_DIAG_DOUBLE bit 65536), summed; [7] counts the tiles
// (spread over 1024 slots by block so the counters do not contend)
__device__ unsigned long long g_rot_phase[1024 * 8];
#define UPH_ROT_T(k)                                                         \
  if (UPH_DIAG_BITS(diag, 65536) && threadIdx.x == 0) {                     \
    const unsigned long long tn = wall_clock64();                            \
    atomicAdd(&g_rot_phase[8 * (blockIdx.x & 1023) + (k)], tn - tprev);      \
    tprev = tn;                                                              \
  }
#else
#define UPH_ROT_T(k)
#endif
template <bool LOOP>
__global__ void __launch_bounds__(kRFT, UPH_ROT_MINB) k_rotate_cubic_g8f(PlaneRef src, PlaneRef dst,
                                                               const RotateArgs* args,
                                                               int max_rows, int cls_rows,
                                                               int diag,
                                                               uint32_t m_gxy, uint32_t m_gx,
                                                               int loop_count, int tgx, int tgy,
                                                               uint32_t* colsum, int64_t cs_stride) {
  // dynamic LDS: window [max_rows][kRFS] floats, nw[max_rows] u64, then one
  // (kRFH / 8) x kRFW byte output buffer per wave
  extern __shared__ __attribute__((aligned(16))) float winf[];
  __shared__ int32_t win_s[4];
  // colsum (optional): the output's column sums over all rows, added into
  // colsum[s * cs_stride + x] (the next mask scan's, masks.c:54-209), so that
  // scan need not read the rotated plane again; per tile summed in LDS, then
  // one atomic per column
  __shared__ uint32_t csum_s[kRFW];
#if UPH_ROT_V2
  __shared__ int32_t done_s;  // waves whose column sums are in csum_s
#endif
  // one tile (txi, tyi) of sheet s; every return is block-uniform
  auto tile = [&](int txi, int tyi, int s) {
#ifdef UPHIP_DIAG
  unsigned long long tprev = wall_clock64();
#endif
  // the plane selectors and the arguments are loaded together (one round trip)
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const RotateArgs a = args[s];
  if (!a.active) return;
  if (cls_rows != 0) {
    // two launches split the sheets by the window rows their angle needs
    // (cls_rows > 0: at most cls_rows; < 0: more than -cls_rows)
    const int need = kRFH + (int)ceilf((kRFW - 1) * fabsf(a.sinval)) + 5;
    if (cls_rows > 0 ? need > cls_rows : need <= -cls_rows) return;
  }
  const Planes& P = src.P;
  const Rect nm = normalize(a.mask);
  const int32_t sw = nm.x1 - nm.x0 + 1, sh = nm.y1 - nm.y0 + 1;
  const float scx = nm.x0 + sw / 2.0f, scy = nm.y0 + sh / 2.0f;  // primitives.c:137-145
  const float tcx = 0 + sw / 2.0f, tcy = 0 + sh / 2.0f;
  const int32_t tx0 = txi * kRFW, ty0 = tyi * kRFH;
  const int32_t u0 = imax(tx0, 0) - a.mask.x0, u1 = imin(tx0 + kRFW, P.W) - 1 - a.mask.x0;
  const int32_t v0 = imax(ty0, 0) - a.mask.y0, v1 = imin(ty0 + kRFH, P.H) - 1 - a.mask.y0;
  const int32_t cu0 = imax(u0, 0), cu1 = imin(u1, sw - 1);
  const int32_t cv0 = imax(v0, 0), cv1 = imin(v1, sh - 1);
  // the tile's column sums (colsum): zeroed here, added per row below
  auto csum_flush = [&]() {
    __syncthreads();
    if (threadIdx.x < kRFW && tx0 + (int)threadIdx.x < P.W)
      atomicAdd(colsum + s * cs_stride + tx0 + threadIdx.x, csum_s[threadIdx.x]);
  };
#if UPH_ROT_V2
  const bool inside = cu0 <= cu1 && cv0 <= cv1;  // uniform
  if (colsum) {
    if (threadIdx.x < kRFW) csum_s[threadIdx.x] = 0;
    if (threadIdx.x == 0) done_s = 0;
    if (!inside) __syncthreads();  // in-mask tiles: the staging barrier orders it
  }
#else
  // the tile's column sums zeroed; in-mask tiles need no barrier of their
  // own here (the corners barrier below orders these writes before any
  // wave's adds), so wave 0 starts on the corners while the block's other
  // waves are still arriving
  const bool outside_tile = !(cu0 <= cu1 && cv0 <= cv1);
  if (colsum) {
    if (threadIdx.x < kRFW) csum_s[threadIdx.x] = 0;
    if (!UPH_ROT_EARLY || outside_tile) __syncthreads();
  }
#endif
  if (!(cu0 <= cu1 && cv0 <= cv1)) {
    // no pixel of the tile inside the mask: copied unchanged (deskew.c:268-286)
    const int cb = 8 * (threadIdx.x & 15);
    const int32_t x = tx0 + cb;
    uint32_t cs8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = threadIdx.x >> 4; r < kRFH; r += kRFT / 16) {
      const int32_t y = ty0 + r;
      if (y >= P.H || x >= P.W) continue;
      const uint8_t* sp = sbase + row_off(y, P.pitch) + x;
      uint8_t* dp = dbase + row_off(y, P.pitch) + x;
      if (x + 8 <= P.W) {
        const uint64_t q = *reinterpret_cast<const uint64_t*>(sp);
        *reinterpret_cast<uint64_t*>(dp) = q;
#pragma unroll
        for (int j = 0; j < 8; j++) cs8[j] += (uint32_t)(q >> (8 * j)) & 0xFFu;
      } else {
        for (int j = 0; x + j < P.W; j++) {
          dp[j] = sp[j];
          cs8[j & 7] += sp[j];
        }
      }
    }
    if (colsum) {
#pragma unroll
      for (int j = 0; j < 8; j++) atomicAdd(&csum_s[cb + j], cs8[j]);
      csum_flush();
    }
    return;
  }
  UPH_ROT_T(0)
  const int lane = threadIdx.x & 63;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Source window of the tile's in-mask pixels (their 4x4 taps included).
  // Every pixel's coordinate lies between the corners' (the same float
  // expression, monotone in u and v); its taps span (int)c - 1 .. (int)c + 2,
  // and (int)c <= floor(c) + 1 (truncation of negatives).  The window is a
  // per-tile constant: wave 0 evaluates the four corners in lanes (c = lane
  // & 3), reduces them across the quad and posts the bounds in LDS, instead
  // of every wave running the float chain of all four corners.
#if UPH_ROT_V2
  // every wave: the corners in lanes (c = lane & 3), reduced across the quad;
  // lane 0's quad holds the bounds (no LDS round trip, no barrier)
  int32_t bx0, by0, bw, bh;
  {
    const int c = lane & 3;
    const int32_t u = c & 1 ? cu1 : cu0, v = c & 2 ? cv1 : cv0;
    const float X = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
    const float Y = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
    float mnx = fminf(X, dpp_f<0xB1>(X)), mxx = fmaxf(X, dpp_f<0xB1>(X));
    float mny = fminf(Y, dpp_f<0xB1>(Y)), mxy = fmaxf(Y, dpp_f<0xB1>(Y));
    mnx = fminf(mnx, dpp_f<0x4E>(mnx));
    mxx = fmaxf(mxx, dpp_f<0x4E>(mxx));
    mny = fminf(mny, dpp_f<0x4E>(mny));
    mxy = fmaxf(mxy, dpp_f<0x4E>(mxy));
    bx0 = __builtin_amdgcn_readfirstlane((int32_t)floorf(mnx)) - 1;
    by0 = __builtin_amdgcn_readfirstlane((int32_t)floorf(mny)) - 1;
    bw = __builtin_amdgcn_readfirstlane((int32_t)floorf(mxx)) + 3 - bx0 + 1;
    bh = __builtin_amdgcn_readfirstlane((int32_t)floorf(mxy)) + 3 - by0 + 1;
  }
  UPH_ROT_T(1)
#else
  if (wu == 0) {
    const int c = lane & 3;
    const int32_t u = c & 1 ? cu1 : cu0, v = c & 2 ? cv1 : cv0;
    const float X = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
    const float Y = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
    float mnx = fminf(X, dpp_f<0xB1>(X)), mxx = fmaxf(X, dpp_f<0xB1>(X));
    float mny = fminf(Y, dpp_f<0xB1>(Y)), mxy = fmaxf(Y, dpp_f<0xB1>(Y));
    mnx = fminf(mnx, dpp_f<0x4E>(mnx));
    mxx = fmaxf(mxx, dpp_f<0x4E>(mxx));
    mny = fminf(mny, dpp_f<0x4E>(mny));
    mxy = fmaxf(mxy, dpp_f<0x4E>(mxy));
    if (lane < 4) {
      const float q = lane == 0 ? mnx : lane == 1 ? mny : lane == 2 ? mxx : mxy;
      win_s[lane] = (int32_t)floorf(q);
    }
  }
  __syncthreads();
  UPH_ROT_T(1)
  const int32_t bx0 = __builtin_amdgcn_readfirstlane(win_s[0]) - 1;
  const int32_t by0 = __builtin_amdgcn_readfirstlane(win_s[1]) - 1;
  const int32_t bw = __builtin_amdgcn_readfirstlane(win_s[2]) + 3 - bx0 + 1;
  const int32_t bh = __builtin_amdgcn_readfirstlane(win_s[3]) + 3 - by0 + 1;
#endif
  const int32_t xa = bx0 >= 0 ? (bx0 & ~3) : -((-bx0 + 3) & ~3);  // window start, dword aligned
  const int nd = (bx0 - xa + bw + 3) >> 2;                         // source dwords per row
  const bool staged = bw > 0 && bh > 0 && 4 * nd <= kRFS && bh <= max_rows;
  uint64_t* nw = reinterpret_cast<uint64_t*>(winf + kRFS * max_rows);
  uint8_t* obuf = reinterpret_cast<uint8_t*>(nw + max_rows) + wu * (kRFH / kRFWaves * kRFW);
  if (staged && !UPH_DIAG_BITS(diag, 1024)) {
    // A wave-instruction stages three window rows, 8 bytes per lane: lanes
    // 18 q .. 18 q + 17 load row r + q (q < 3), lanes 54..63 idle.  nw[r] bit j:
    // window bytes 8 j .. 8 j + 7 of row r hold a non-white pixel.
    const int rq = (lane * 57) >> 10;  // lane / 18 for lane < 64
    const int jq = lane - 18 * rq;
    const int nq = (nd + 1) >> 1;
    const bool qv = rq < 3 && jq < nq;
    const int32_t xd = xa + 8 * jq;
    // one wave-instruction's rows: ballot, non-white flags, fp32 window row
    auto stage = [&](int rb, uint32_t w0, uint32_t w1) {
      const int r = rb + rq;
      const bool valid = qv && r < bh;
      const unsigned long long m = __ballot(valid && (w0 & w1) != 0xFFFFFFFFu);
      if (lane < 3 && rb + lane < bh) nw[rb + lane] = (m >> (18 * lane)) & 0x3FFFFull;
      if (valid) {
        float4* d = reinterpret_cast<float4*>(winf + r * kRFS + 8 * jq);
        d[0] = make_float4(ubyte_f<0>(w0), ubyte_f<1>(w0), ubyte_f<2>(w0), ubyte_f<3>(w0));
        d[1] = make_float4(ubyte_f<0>(w1), ubyte_f<1>(w1), ubyte_f<2>(w1), ubyte_f<3>(w1));
      }
    };
    const bool interior = xa >= 0 && xa + 8 * nq <= P.W && by0 >= 0 && by0 + bh <= P.H;
    if (interior) {
      // the whole window inside the image: straight loads.  A lane's byte
      // offset is its row-rq offset plus a scalar row product per group;
      // lanes past the window's rows (and idle lanes) read their row rq.
      const uint32_t off0 = row_off(by0 + rq, P.pitch) + (uint32_t)(qv ? xd : xa);
      for (int rg = 3 * wu; rg < bh; rg += 3 * 3 * kRFWaves) {
        uint2 v[3];
#pragma unroll
        for (int g = 0; g < 3; g++) {  // all loads of the group in flight
          const int rb = rg + 3 * kRFWaves * g;
          const uint32_t o = rb + rq < bh ? off0 + (uint32_t)rb * (uint32_t)P.pitch : off0;
          v[g] = *reinterpret_cast<const uint2*>(sbase + o);
        }
#pragma unroll
        for (int g = 0; g < 3; g++) {
          const int rb = rg + 3 * kRFWaves * g;  // the wave's first row of this instruction
          if (rb >= bh) break;                   // uniform
          stage(rb, v[g].x, v[g].y);
        }
      }
    } else {
      // edge tiles load every dword clamped into the row, realign it by one
      // 64-bit shift and make the bytes outside [0, W) x [0, H) white
      const int32_t xc0 = imin(imax(xd, 0), (int32_t)P.pitch - 4);
      const int32_t xc1 = imin(imax(xd + 4, 0), (int32_t)P.pitch - 4);
      const int fs0 = imin(imax(24 + 8 * (xd - xc0), 0), 56);
      const int fs1 = imin(imax(24 + 8 * (xd + 4 - xc1), 0), 56);
      uint32_t out0 = qv ? 0u : 0xFFFFFFFFu, out1 = out0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (xd + k < 0 || xd + k >= P.W) out0 |= 0xFFu << (8 * k);
        if (xd + 4 + k < 0 || xd + 4 + k >= P.W) out1 |= 0xFFu << (8 * k);
      }
      for (int rg = 3 * wu; rg < bh; rg += 3 * 3 * kRFWaves) {
        uint2 v[3];
#pragma unroll
        for (int g = 0; g < 3; g++) {
          const int r = rg + 3 * kRFWaves * g + rq;
          const int32_t y = imin(imax(by0 + r, 0), P.H - 1);
          const uint8_t* row = sbase + row_off(y, P.pitch);
          v[g].x = *reinterpret_cast<const uint32_t*>(row + xc0);
          v[g].y = *reinterpret_cast<const uint32_t*>(row + xc1);
        }
#pragma unroll
        for (int g = 0; g < 3; g++) {
          const int rb = rg + 3 * kRFWaves * g;
          if (rb >= bh) break;
          const int32_t y = by0 + rb + rq;
          uint32_t w0 = (uint32_t)(((uint64_t)v[g].x << 24) >> fs0) | out0;
          uint32_t w1 = (uint32_t)(((uint64_t)v[g].y << 24) >> fs1) | out1;
          if ((y < 0) | (y >= P.H)) w0 = w1 = 0xFFFFFFFFu;
          stage(rb, w0, w1);
        }
      }
    }
  }
  __syncthreads();
  UPH_ROT_T(2)
  const int32_t xA = tx0 + lane, xB = xA + 64;
  const bool hasA = xA < P.W, hasB = xB < P.W;
  // per-lane terms of the source coordinates (constant down the column):
  //   srcX = (scx + (u - tcx) cos) + (v - tcy) sin
  //   srcY = (scy + (v - tcy) cos) - (u - tcx) sin
  const int32_t uA = xA - a.mask.x0, uB = xB - a.mask.x0;
  const float cuA = uA - tcx, cuB = uB - tcx;
  const float axA = scx + cuA * a.cosval, bsA = cuA * a.sinval;
  const float axB = scx + cuB * a.cosval, bsB = cuB * a.sinval;
  const bool colA = hasA & (uA >= 0) & (uA < sw), colB = hasB & (uB >= 0) & (uB < sw);
  typedef __attribute__((address_space(3))) float lds_f32;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_f32*)winf;  // LDS byte address of winf
  const Src<F_GRAY8> S{sbase, P.pitch, P.W, P.H};
  // Source coordinates are monotone along a row, so the tap rows of all 128
  // columns of a tile row lie between those of its end columns (computed
  // with the same expressions, wave-uniform).  When every tap there is white
  // (255) the bicubic result is exactly 255: all differences are zero, so
  // each cubic_scale returns b + (+-0) = b.
  const float cuL = (tx0 - a.mask.x0) - tcx, cuR = (tx0 + kRFW - 1 - a.mask.x0) - tcx;
  const float bsL = cuL * a.sinval, bsR = cuR * a.sinval;
  constexpr int kRows = kRFH / kRFWaves;            // rows per wave
  const int32_t yw = ty0 + wu * kRows;              // the wave's rows: yw .. yw + kRows-1
  // Outside the mask a pixel is copied unchanged (deskew.c:268-286).  Those
  // source bytes are read into the wave's output buffer first: on gfx9 a
  // wait for a load also waits for every earlier store, so no global load
  // may follow the first store.  Tiles wholly inside the mask skip this.
  // The wave's output rows move through obuf with one mapping for loads and
  // stores: lane -> row k0 + lane/16, bytes 8*(lane%16), k0 = 0, 4.
  const int cb = 8 * (lane & 15);
  const int32_t xo = tx0 + cb;
  const bool partial = !(cu0 == u0 && cu1 == u1 && cv0 == v0 && cv1 == v1);
  if (partial) {
    constexpr int kQ = (kRows + 3) / 4;
    uint64_t q[kQ];
#pragma unroll
    for (int h = 0; h < kQ; h++) {
      q[h] = 0;
      const int rr = 4 * h + (lane >> 4);
      const int32_t y = imin(yw + rr, P.H - 1);
      const int32_t x = imin(xo, (int32_t)P.pitch - 8);  // rows are 256-byte pitched
      if (rr < kRows) q[h] = *reinterpret_cast<const uint64_t*>(sbase + row_off(y, P.pitch) + x);
    }
#pragma unroll
    for (int h = 0; h < kQ; h++) {
      const int rr = 4 * h + (lane >> 4);
      if (rr < kRows) *reinterpret_cast<uint64_t*>(obuf + rr * kRFW + cb) = q[h];
    }
  }
  // White flags of the wave's rows, computed lane-parallel up front: lane
  // 16 q + j tests window row r0 + j (+16, ...) of output row 4 h + q against
  // the row's dword columns; one ballot per four rows (instead of scalar
  // bounds and a ballot per row).
  uint32_t white_rows = 0;  // bit k: every tap of output row k is white
  if (staged) {
    // one pass: lane 8 k + j tests output row k against window rows
    // r0 + j, r0 + j + 8, ... of the row's tap band, over the whole window
    // width (a row's taps span all but the ~(kRFH sin) columns of the
    // window's slant, so a column restriction would rarely change a flag)
#pragma unroll
    for (int g = 0; g < kRows; g += 8) {
      const int k = g + (lane >> 3), j = lane & 7;
      bool hit = false;
      if (k < kRows) {
        const float cv = (yw + k - a.mask.y0) - tcy;
        const float VC = scy + cv * a.cosval;
        const int32_t yl = (int)(VC - bsL), yr = (int)(VC - bsR);
        const int32_t r0 = imax(imin(yl, yr) - 1 - by0, 0);
        const int32_t r1 = imin(imax(yl, yr) + 2 - by0, bh - 1);
        for (int r = r0 + j; r <= r1; r += 8) hit |= nw[r] != 0;
      }
      const uint64_t m = __ballot(hit);
#pragma unroll
      for (int q = 0; q < 8 && g + q < kRows; q++)
        if (((m >> (8 * q)) & 0xFFull) == 0) white_rows |= 1u << (g + q);
    }
    if (UPH_DIAG_BITS(diag, 2048)) white_rows = 0;
    if (UPH_DIAG_BITS(diag, 512)) white_rows = ~0u;
  }
  // Every source coordinate of the tile's in-mask pixels is >= 1 when the
  // window starts inside the image: then (int)c == floor(c) and
  // c - (int)c == fract(c) exactly (one instruction instead of three).
  const bool posc = bx0 >= 0 && by0 >= 0;
  // LDS byte address of window (row 0, column 0) minus the 4x4 tap offset,
  // so a pixel's first tap sits at wbase + 4 (iy kRFS + ix)
  const uint32_t wbase = lds0 - 4u * (uint32_t)((1 + by0) * kRFS + 1 + xa);
  UPH_ROT_T(3)
  // Full tiles (every pixel inside the mask and the image, the window staged
  // and starting inside the image) take a copy of the row loop without the
  // per-pixel mask tests and their exec-mask branches.
  uint32_t fsA = 0, fsB = 0;  // full tiles: this wave's column sums
  auto row_loop = [&](auto full_tag) {
  constexpr bool FULL = decltype(full_tag)::value;
#pragma unroll
  for (int k = 0; k < kRows; k++) {
    const int32_t y = yw + k;
    const int32_t v = y - a.mask.y0;
    const bool rowin = FULL || ((v >= 0) & (v < sh) & (y < P.H));
    const float cv = v - tcy;
    const float VS = cv * a.sinval, VC = scy + cv * a.cosval;
    const bool inA = FULL || (rowin & colA), inB = FULL || (rowin & colB);
    uint32_t oA = 255, oB = 255;
    const bool white = (FULL || staged) && ((white_rows >> k) & 1u);
    if (!white && (FULL || staged)) {
      const float sxA = axA + VS, syA = VC - bsA, sxB = axB + VS, syB = VC - bsB;
      const int ixA = (int)sxA, iyA = (int)syA, ixB = (int)sxB, iyB = (int)syB;  // truncation
      float fxA, fyA, fxB, fyB;
      if (FULL || posc) {
        fxA = __builtin_amdgcn_fractf(sxA);
        fyA = __builtin_amdgcn_fractf(syA);
        fxB = __builtin_amdgcn_fractf(sxB);
        fyB = __builtin_amdgcn_fractf(syB);
      } else {
        fxA = sxA - ixA, fyA = syA - iyA, fxB = sxB - ixB, fyB = syB - iyB;
      }
      // window address as one full-rate 24-bit multiply-add; pixels outside
      // the mask read (and discard) the window origin
      const uint32_t pA = inA ? wbase + 4u * (uint32_t)(__mul24(iyA, kRFS) + ixA) : lds0;
      const uint32_t pB = inB ? wbase + 4u * (uint32_t)(__mul24(iyB, kRFS) + ixB) : lds0;
      const uint32_t ta[4] = {pA, pA + 8 * kRFS, pB, pB + 8 * kRFS};
      f2 t[4][4];
      lds_taps16(ta, t);
#if UPH_ROT_UNIFORM
      // A/B variant: a wave row whose every pixel has a
      // uniform 4x4 window (all taps equal: every difference is 0, so each
      // cubic_scale returns its b) skips the arithmetic
      lds_wait_pair<0>(t[3]);
      bool uni = true;
#pragma unroll
      for (int pp = 0; pp < 4; pp++)
#pragma unroll
        for (int j = 0; j < 4; j++)
          uni = uni && t[pp][j].x == t[pp & 2][0].x && t[pp][j].y == t[pp & 2][0].x;
      if (__builtin_amdgcn_ballot_w64(!uni) == 0) {
        oA = (uint32_t)t[0][0].x;
        oB = (uint32_t)t[2][0].x;
      } else
#endif
      {
      // rows (0,1) and (2,3) of A once its eight tap pairs are in, then of B
      const f2 FA = splat2(fxA), HA = splat2(0.5f * fxA);
      const f2 FB = splat2(fxB), HB = splat2(0.5f * fxB);
      f2 c[4];  // unclamped row results; clamped straight into the column pairs
#if UPH_ROT_PAIRS
      // A's two row pairs interleaved once its eight tap pairs are in, then B's
      lds_wait_pairs<8>(t[0], t[1]);
      cubic2_row_u2(FA, HA, t[0], FA, HA, t[1], c[0], c[1]);
      lds_wait_pairs<0>(t[2], t[3]);
      cubic2_row_u2(FB, HB, t[2], FB, HB, t[3], c[2], c[3]);
#else
      lds_wait_pair<12>(t[0]);
      c[0] = cubic2_row_u(FA, HA, t[0]);
      lds_wait_pair_after<8>(t[1], c[0]);
      c[1] = cubic2_row_u(FA, HA, t[1]);
      lds_wait_pair_after<4>(t[2], c[1]);
      c[2] = cubic2_row_u(FB, HB, t[2]);
      lds_wait_pair_after<0>(t[3], c[2]);
      c[3] = cubic2_row_u(FB, HB, t[3]);
#endif
      // the column cubic of A and B as one pair
      const f2 o = cubic2(f2{fyA, fyB}, f2{0.5f * fyA, 0.5f * fyB},
                          f2{clamp_t255(c[0].x), clamp_t255(c[2].x)},
                          f2{clamp_t255(c[0].y), clamp_t255(c[2].y)},
                          f2{clamp_t255(c[1].x), clamp_t255(c[3].x)},
                          f2{clamp_t255(c[1].y), clamp_t255(c[3].y)});
      oA = (uint32_t)o.x;  // integer-valued in [0, 255]
      oB = (uint32_t)o.y;
      }
    }
#ifdef UPHIP_DIAG
    if (UPH_DIAG_BITS(diag, 131072)) {  // tuning: +32 SALU a row (is the scalar unit a limit?)
      int32_t z = k;
      asm volatile(
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1"
          : "+s"(z));
      if (z == -1) oA = 0;
    }
#endif
    if (!FULL && !staged) break;  // uniform: the rows go through the loop below
    if (FULL) {  // every pixel in the mask: no per-lane branches
      obuf[k * kRFW + lane] = (uint8_t)oA;
      obuf[k * kRFW + 64 + lane] = (uint8_t)oB;
      fsA += oA;  // the column sums from registers (no re-read of obuf)
      fsB += oB;
    } else {
      if (inA) obuf[k * kRFW + lane] = (uint8_t)oA;
      if (inB) obuf[k * kRFW + 64 + lane] = (uint8_t)oB;
    }
  }
  };
  const bool full =
      UPH_ROT_FULL && !partial && staged && posc && tx0 + kRFW <= P.W && ty0 + kRFH <= P.H;
  if (full)
    row_loop(std::true_type{});
  else
    row_loop(std::false_type{});
  if (!staged) {
    // window too large for LDS (large angles): taps from the frame (kept out
    // of the unrolled loop above)
#pragma unroll 1
    for (int k = 0; k < kRows; k++) {
      const int32_t y = yw + k;
      const int32_t v = y - a.mask.y0;
      const bool rowin = (v >= 0) & (v < sh) & (y < P.H);
      const float cv = v - tcy;
      const float VS = cv * a.sinval, VC = scy + cv * a.cosval;
      if (rowin & colA) obuf[k * kRFW + lane] = interp_bicubic(S, axA + VS, VC - bsA).r;
      if (rowin & colB) obuf[k * kRFW + 64 + lane] = interp_bicubic(S, axB + VS, VC - bsB).r;
    }
  }
  UPH_ROT_T(4)
  // the wave's rows as 8-byte stores: lane -> row k0 + lane/16, bytes
  // 8*(lane%16).  One wave's LDS operations complete in order, so its reads
  // see its writes without a fence.
  __builtin_amdgcn_wave_barrier();
  if (full && !UPH_DIAG_BITS(diag, 8192)) {
    // inside the image: no bounds tests
#pragma unroll
    for (int k0 = 0; k0 < kRows; k0 += 4) {
      const int rr = k0 + (lane >> 4);
      if (rr < kRows) {
        const uint64_t q = *reinterpret_cast<const uint64_t*>(obuf + rr * kRFW + cb);
        *reinterpret_cast<uint64_t*>(dbase + row_off(yw + rr, P.pitch) + xo) = q;
      }
    }
  } else
  for (int k0 = 0; k0 < kRows && !UPH_DIAG_BITS(diag, 8192); k0 += 4) {
    const int rr = k0 + (lane >> 4);
    const int32_t y = yw + rr, x = xo;
    if (rr < kRows && y < P.H && x < P.W) {
      const uint64_t q = *reinterpret_cast<const uint64_t*>(obuf + rr * kRFW + cb);
      uint8_t* d = dbase + row_off(y, P.pitch) + x;
      if (x + 8 <= P.W) {
        *reinterpret_cast<uint64_t*>(d) = q;
      } else {
        for (int j = 0; x + j < P.W; j++) d[j] = (uint8_t)(q >> (8 * j));
      }
    }
  }
  UPH_ROT_T(5)
  if (colsum) {
    // this wave's rows of columns lane and 64 + lane, then the tile's
    uint32_t sA = fsA, sB = fsB;
    if (!full) {
#pragma unroll
      for (int k = 0; k < kRows; k++) {
        if (yw + k >= P.H) break;
        sA += obuf[k * kRFW + lane];
        sB += obuf[k * kRFW + 64 + lane];
      }
    }
#if UPH_ROT_V2
    // the wave's sums into the tile's, then the last wave to arrive adds the
    // tile's into the sheet's (release/acquire on the arrival counter orders
    // every wave's LDS adds before the last wave's reads)
    __hip_atomic_fetch_add(&csum_s[lane], sA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(&csum_s[64 + lane], sB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    int prev = 0;
    if (lane == 0)
      prev = __hip_atomic_fetch_add(&done_s, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev = __shfl(prev, 0, 64);
    if (prev == kRFWaves - 1) {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);
      uint32_t* cs = colsum + s * cs_stride + tx0;
      const uint32_t vA = __hip_atomic_load(&csum_s[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint32_t vB = __hip_atomic_load(&csum_s[64 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (tx0 + lane < P.W) atomicAdd(cs + lane, vA);
      if (tx0 + 64 + lane < P.W) atomicAdd(cs + 64 + lane, vB);
    }
#else
    atomicAdd(&csum_s[lane], sA);
    atomicAdd(&csum_s[64 + lane], sB);
    csum_flush();
#endif
  }
  UPH_ROT_T(6)
#ifdef UPHIP_DIAG
  if (UPH_DIAG_BITS(diag, 65536) && threadIdx.x == 0)
    atomicAdd(&g_rot_phase[8 * (blockIdx.x & 1023) + 7], 1ull);
#endif
  };
  if constexpr (!LOOP) {  // one tile per block, XCD-aware order
    int txi, tyi, s;
    xcd_block_m(m_gxy, m_gx, &txi, &tyi, &s);
    tile(txi, tyi, s);
  } else {
  // Persistent form for the large-window class, usually empty: the lanes of
  // every wave test 64 sheets at once (the same ballot in every wave), and
  // the block walks the tiles of the sheets that belong here.
  for (int s0 = 0; s0 < loop_count; s0 += 64) {
    const int l = threadIdx.x & 63;
    bool want = false;
    if (s0 + l < loop_count) {
      const RotateArgs q = args[s0 + l];
      want = q.active && kRFH + (int)ceilf((kRFW - 1) * fabsf(q.sinval)) + 5 > -cls_rows;
    }
    uint64_t m = __ballot(want);
    m = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(m >> 32)) << 32) |
        __builtin_amdgcn_readfirstlane((uint32_t)m);
    while (m) {
      const int s = s0 + __ffsll((long long)m) - 1;
      m &= m - 1;
      for (int t = blockIdx.x; t < tgx * tgy; t += gridDim.x) {
        tile(t % tgx, t / tgx, s);
        __syncthreads();  // the next tile restages the LDS window
      }
    }
  }
  }
}

// Rows of source window a kRFW x kRFH tile needs at rotations up to |angle|.
static int rotate_window_rows(float max_abs_angle) {
  const float a = fminf(fabsf(max_abs_angle), 1.5707964f);
  // (kRFH-1) cos + (kRFW-1) sin rows of pixel centres, + 3 tap rows, + 2 for
  // the floor/truncation slack of the window bounds
  return kRFH + (int)ceilf((kRFW - 1) * sinf(a)) + 5;
}

bool launch_rotate_mask(const PlaneRef& src, const PlaneRef& dst, const RotateArgs* args,
                        int interp, int count, hipStream_t st, float max_abs_angle,
                        uint32_t* colsum, int64_t cs_stride) {
  const dim3 grid((src.P.W + kRotTW - 1) / kRotTW, (src.P.H + kRotTH - 1) / kRotTH, count);
  const dim3 ggrid((src.P.W + kRotTW - 1) / kRotTW, (src.P.H + kRotGH - 1) / kRotGH, count);
  if (interp == UPHIP_INTERP_CUBIC && src.P.fmt == F_GRAY8) {
    if (diag_double() & 4096) colsum = nullptr;  // tuning build: time without the column sums
    const int rows = rotate_window_rows(max_abs_angle);
    auto lds_of = [](int r) {
      return (sizeof(float) * kRFS + sizeof(uint64_t)) * (size_t)r + kRFH * kRFW;
    };
    // the most window rows that still let four tiles (32 waves) share a CU's
    // 160 KB of LDS (16 + 512 B of static LDS per tile); windows of up to ~2.4 deg
    // (TALL: two tiles, 16 waves, per CU)
    const int rows4 = (int)(((UPH_ROT_TALL ? 80 : 40) * 1024 - 16 - 4 * kRFW - kRFH * kRFW) /
                            (sizeof(float) * kRFS + sizeof(uint64_t)));
    if (UPH_ROT_TALL) {
      allow_dynamic_lds((const void*)k_rotate_cubic_g8f<false>, 120 * 1024);
      allow_dynamic_lds((const void*)k_rotate_cubic_g8f<true>, 120 * 1024);
    }
    if (lds_of(rows) <= (UPH_ROT_TALL ? 120 : 56) * 1024 &&
        src.P.pitch * (int64_t)src.P.H < (1ll << 31) && !(diag_double() & 256)) {
      const dim3 fgrid((src.P.W + kRFW - 1) / kRFW, (src.P.H + kRFH - 1) / kRFH, count);
      const uint32_t mgxy = div_magic(fgrid.x * fgrid.y), mgx = div_magic(fgrid.x);
      const int dd = diag_double() & (512 | 1024 | 2048 | 8192 | 65536 | 131072);
#ifdef UPHIP_DIAG
      struct PhasePrint {  // after the launches below: the per-tile phase clocks
        hipStream_t st;
        ~PhasePrint() {
          if (!(diag_double() & 65536)) return;
          static unsigned long long hh[1024 * 8], z[1024 * 8];
          unsigned long long h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          hipStreamSynchronize(st);
          hipMemcpyFromSymbol(hh, HIP_SYMBOL(g_rot_phase), sizeof(hh));
          hipMemcpyToSymbol(HIP_SYMBOL(g_rot_phase), z, sizeof(z));
          for (int i = 0; i < 1024 * 8; i++) h[i & 7] += hh[i];
          if (!h[7]) return;
          fprintf(stderr, "rotate phases (10 ns ticks/tile, %llu tiles): args %.0f corners %.0f staging %.0f "
                  "flags %.0f compute %.0f stores %.0f colsum %.0f\n", h[7], (double)h[0] / h[7],
                  (double)h[1] / h[7], (double)h[2] / h[7], (double)h[3] / h[7],
                  (double)h[4] / h[7], (double)h[5] / h[7], (double)h[6] / h[7]);
        }
      } phase_print{st};
#endif
      if (rows > rows4) {
        // sheets whose angle fits the small window at four tiles per CU, then
        // the others at the scan range's window (three per CU); every sheet
        // is taken by exactly one of the two launches
        // (the second as a persistent grid: when no sheet needs the large
        // window its blocks only read the arguments)
        UPH_LAUNCH_DIAG(2, k_rotate_cubic_g8f<false>, fgrid, dim3(kRFT), lds_of(rows4), st, src, dst, args,
                        rows4, rows4, dd, mgxy, mgx, 0, 0, 0, colsum, cs_stride);
        UPH_LAUNCH_DIAG(2, k_rotate_cubic_g8f<true>, dim3(3 * 256), dim3(kRFT), lds_of(rows), st, src, dst,
                        args, rows, -rows4, dd, 0u, 0u, count, (int)fgrid.x, (int)fgrid.y, colsum,
                        cs_stride);
      } else {
        UPH_LAUNCH_DIAG(2, k_rotate_cubic_g8f<false>, fgrid, dim3(kRFT), lds_of(rows), st, src, dst, args,
                        rows, 0, dd, mgxy, mgx, 0, 0, 0, colsum, cs_stride);
      }
      return colsum != nullptr;
    }
    const dim3 qgrid((src.P.W + kRQW - 1) / kRQW, (src.P.H + kRQH - 1) / kRQH, count);
    UPH_LAUNCH_DIAG(2, k_rotate_cubic_g8, qgrid, dim3(kThreads), 0, st, src, dst, args);
    return false;
  }
  if (interp == UPHIP_INTERP_CUBIC && src.P.fmt == F_Y400A) {
    hipLaunchKernelGGL(k_rotate_cubic_gray<F_Y400A>, ggrid, dim3(kThreads), 0, st, src, dst, args);
    return false;
  }
  if (src.P.fmt == F_GRAY8)
    hipLaunchKernelGGL(k_rotate_mask<F_GRAY8>, grid, dim3(kThreads), 0, st, src, dst, args,
                       interp);
  else if (src.P.fmt == F_Y400A)
    hipLaunchKernelGGL(k_rotate_mask<F_Y400A>, grid, dim3(kThreads), 0, st, src, dst, args,
                       interp);
  else
    hipLaunchKernelGGL(k_rotate_mask<F_RGB24>, grid, dim3(kThreads), 0, st, src, dst, args,
                       interp);
  return false;
}

__global__ void k_flip_if_active(SheetCtl* ctl, const int32_t* active, int64_t stride_ints,
                                 int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < count && active[(int64_t)s * stride_ints]) ctl[s].cur ^= 1;
}

void launch_flip_if_active(SheetCtl* ctl, const int32_t* active, int64_t stride_bytes, int count,
                           hipStream_t st) {
  hipLaunchKernelGGL(k_flip_if_active, dim3((count + 255) / 256), dim3(256), 0, st, ctl, active,
                     stride_bytes / 4, count);
}

}  // namespace uph
