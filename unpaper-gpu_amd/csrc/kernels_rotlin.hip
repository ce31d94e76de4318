// kernels_rotlin.hip — deskew rotation with bilinear interpolation
// (deskew.c:248-286 + interp_bilinear, interpolate.c:76-117): the --interpolate
// linear path, BASELINE configs[3]'s RGB24 double-page scans.
//
// One workgroup per 64 x 32 output tile, one output pixel per lane and row.
// The tile's source window is staged once in LDS as C float planes (one per
// channel; white outside the image, which is get_pixel's value there), so the
// four taps of a channel are two ds_read2_b32.  Red and green run as packed
// pairs, every rounding of linear_scale kept:  (uint8)((1.0f - x) * a + x * b).
// Output rows are assembled in LDS (pixels outside every rotated mask keep the
// source bytes) and leave as 16-byte stores.
//
// Up to two masks per sheet in one launch (the double layout): mask 1 is
// rotated here only when the caller marked the sheet independent -- its
// rotation was detected on the same image and its source window does not reach
// into mask 0 (k_rot_independent) -- so the result equals the reference's
// one-mask-after-the-other order (sheet_stages.c:401-412); otherwise mask 1
// takes a second launch after mask 0's.
#include "interp.h"
#include "kernels.h"

namespace uph {

typedef float lf2 __attribute__((ext_vector_type(2)));

// byte K of w as a float (one v_cvt_f32_ubyteK)
template <int K>
__device__ __forceinline__ float ubyte_f(uint32_t w) {
  return (float)((w >> (8 * K)) & 0xFFu);
}

constexpr int kLW = 64;                    // output columns per tile (one per lane)
constexpr int kLH = 32;                    // output rows per tile
constexpr int kLT = 256;                   // 4 waves, kLH / 4 consecutive rows each
constexpr int kLRows = kLH / (kLT / 64);

// linear_scale (interpolate.c:62-65) on the pair (r, g): separate roundings of
// (1 - x) * a, x * b and their sum, then the uint8 truncation
__device__ __forceinline__ lf2 lin2(float xm, float x, lf2 a, lf2 b) {
  const lf2 t = lf2{xm, xm} * a;
  const lf2 u = lf2{x, x} * b;
  const lf2 s = t + u;
  return lf2{__builtin_truncf(s.x), __builtin_truncf(s.y)};
}
// the same on two pixels, each with its own fraction
__device__ __forceinline__ lf2 lin2v(lf2 xm, lf2 x, lf2 a, lf2 b) {
  const lf2 t = xm * a;
  const lf2 u = x * b;
  const lf2 s = t + u;
  return lf2{__builtin_truncf(s.x), __builtin_truncf(s.y)};
}
__device__ __forceinline__ float lin1(float xm, float x, float a, float b) {
  const float t = xm * a, u = x * b;
  return __builtin_truncf(t + u);
}

// In-mask part of a tile for one mask, in mask coordinates; false when empty.
struct MaskPart {
  int32_t cu0, cu1, cv0, cv1;
  bool full;  // every pixel of the tile lies in the mask
};
__device__ __forceinline__ bool mask_part(const RotateArgs& a, int32_t tx0, int32_t ty0, int32_t W,
                                          int32_t H, MaskPart* mp) {
  const Rect nm = normalize(a.mask);
  const int32_t sw = nm.x1 - nm.x0 + 1, sh = nm.y1 - nm.y0 + 1;
  const int32_t u0 = imax(tx0, 0) - a.mask.x0, u1 = imin(tx0 + kLW, W) - 1 - a.mask.x0;
  const int32_t v0 = imax(ty0, 0) - a.mask.y0, v1 = imin(ty0 + kLH, H) - 1 - a.mask.y0;
  mp->cu0 = imax(u0, 0);
  mp->cu1 = imin(u1, sw - 1);
  mp->cv0 = imax(v0, 0);
  mp->cv1 = imin(v1, sh - 1);
  mp->full = mp->cu0 == u0 && mp->cu1 == u1 && mp->cv0 == v0 && mp->cv1 == v1;
  return mp->cu0 <= mp->cu1 && mp->cv0 <= mp->cv1;
}

template <int FMT>
__global__ void __launch_bounds__(kLT) k_rotate_lin(PlaneRef src, PlaneRef dst, const RotateArgs* args,
                                                    int nmask, int64_t mstride, const int32_t* indep,
                                                    LinWindow win, uint32_t m_gxy, uint32_t m_gx) {
  constexpr int C = FMT == F_RGB24 ? 3 : 1;
  constexpr int kRowB = kLW * C;            // output bytes per tile row
  extern __shared__ __attribute__((aligned(16))) float lw[];  // C planes [rows][stride], then obuf
  __shared__ int32_t wb[4];
  int txi, tyi, s;
  xcd_block_m(m_gxy, m_gx, &txi, &tyi, &s);
  bool on[2] = {false, false};
  RotateArgs am[2];
#pragma unroll
  for (int m = 0; m < 2; m++) {
    if (m >= nmask) break;
    am[m] = args[m * mstride + s];
    on[m] = am[m].active && (m == 0 || !indep || indep[s]);
  }
  if (!on[0] && !on[1]) return;  // not rotated here: the plane is not flipped
  const Planes& P = src.P;
  const uint8_t* sbase = plane_ptr(src, s);
  uint8_t* dbase = plane_ptr(dst, s);
  const int32_t tx0 = txi * kLW, ty0 = tyi * kLH;
  const int32_t th = imin(kLH, P.H - ty0);
  const int64_t xb0 = (int64_t)tx0 * C;                     // tile's first byte in a row
  const int32_t rowb = (int32_t)imin((int64_t)kRowB, (int64_t)P.W * C - xb0);  // its bytes per row
  MaskPart mp[2];
  bool hit[2] = {false, false};
#pragma unroll
  for (int m = 0; m < 2; m++)
    if (on[m]) hit[m] = mask_part(am[m], tx0, ty0, P.W, P.H, &mp[m]);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 16-byte vectors of a tile row that lie inside the row's pitch
  auto vec_ok = [&](int j) { return xb0 + 16 * (j + 1) <= P.pitch; };
  if (!hit[0] && !hit[1]) {
    // no rotated pixel: the tile's bytes copied unchanged (deskew.c:268-286)
    constexpr int NV = kRowB / 16;
    for (int i = tid; i < th * NV; i += kLT) {
      const int r = i / NV, j = i - r * NV;
      if (16 * j >= rowb) continue;
      const uint8_t* sp = sbase + (int64_t)(ty0 + r) * P.pitch + xb0 + 16 * j;
      uint8_t* dp = dbase + (int64_t)(ty0 + r) * P.pitch + xb0 + 16 * j;
      if (vec_ok(j) && 16 * (j + 1) <= rowb) {
        *reinterpret_cast<uint4*>(dp) = *reinterpret_cast<const uint4*>(sp);
      } else {
        for (int k = 0; k < 16 && 16 * j + k < rowb; k++) dp[k] = sp[k];
      }
    }
    return;
  }
  // the window: GRAY8 as floats; RGB24 as one 32-bit word per pixel
  // (r | g << 8 | b << 16), converted per tap -- a third of three float
  // planes' LDS, so eight tiles share a CU instead of three
  const int32_t plane_f = win.rows * win.stride;            // words per window
  uint32_t* lwu = reinterpret_cast<uint32_t*>(lw);
  uint8_t* obuf = reinterpret_cast<uint8_t*>(lw + plane_f);  // kLH x kRowB bytes
  // 1. the tile's source bytes (kept where no mask rotates); a tile wholly
  // inside one rotating mask is overwritten pixel by pixel and skips this
  if (!((hit[0] && mp[0].full) || (hit[1] && mp[1].full))) {
    constexpr int NV = kRowB / 16;
    for (int i = tid; i < th * NV; i += kLT) {
      const int r = i / NV, j = i - r * NV;
      const uint8_t* sp = sbase + (int64_t)(ty0 + r) * P.pitch + xb0 + 16 * j;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (16 * j < rowb) {
        if (vec_ok(j)) {
          v = *reinterpret_cast<const uint4*>(sp);
        } else {  // the row's last bytes, one at a time (no array: it would live in scratch)
          uint32_t wv4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int k = 0; k < 16; k++)
            if (16 * j + k < rowb) wv4[k >> 2] |= (uint32_t)sp[k] << (8 * (k & 3));
          v = make_uint4(wv4[0], wv4[1], wv4[2], wv4[3]);
        }
      }
      *reinterpret_cast<uint4*>(obuf + r * kRowB + 16 * j) = v;
    }
  }
  // 2. every mask that rotates part of the tile (disjoint when both do)
#pragma unroll 1
  for (int m = 0; m < 2; m++) {
    // static indices only (a run-time index would put the arrays in scratch)
    if (!(m == 0 ? hit[0] : hit[1])) continue;
    const RotateArgs a = m == 0 ? am[0] : am[1];
    const MaskPart mpm = m == 0 ? mp[0] : mp[1];
    const Rect nm = normalize(a.mask);
    const int32_t sw = nm.x1 - nm.x0 + 1, sh = nm.y1 - nm.y0 + 1;
    const float scx = nm.x0 + sw / 2.0f, scy = nm.y0 + sh / 2.0f;  // primitives.c:137-145
    const float tcx = 0 + sw / 2.0f, tcy = 0 + sh / 2.0f;
    // source window of the in-mask pixels: coordinates are monotone in u
    // and v (the same float expressions), so the corners bound them; the
    // taps are floor(c) .. ceil(c) <= floor(c) + 1
    if (wv == 0) {
      const int c = lane & 3;
      const int32_t u = c & 1 ? mpm.cu1 : mpm.cu0, v = c & 2 ? mpm.cv1 : mpm.cv0;
      const float X = scx + (u - tcx) * a.cosval + (v - tcy) * a.sinval;
      const float Y = scy + (v - tcy) * a.cosval - (u - tcx) * a.sinval;
      float mnx = X, mxx = X, mny = Y, mxy = Y;
#pragma unroll
      for (int o = 1; o < 4; o <<= 1) {
        mnx = fminf(mnx, __shfl_xor(mnx, o, 64));
        mxx = fmaxf(mxx, __shfl_xor(mxx, o, 64));
        mny = fminf(mny, __shfl_xor(mny, o, 64));
        mxy = fmaxf(mxy, __shfl_xor(mxy, o, 64));
      }
      if (lane < 4) wb[lane] = (int32_t)floorf(lane == 0 ? mnx : lane == 1 ? mny : lane == 2 ? mxx : mxy);
    }
    __syncthreads();
    const int32_t bx0 = wb[0], by0 = wb[1];
    const int32_t bw = wb[2] + 1 - bx0 + 1, bh = wb[3] + 1 - by0 + 1;
    const int32_t bxa = bx0 & ~3;  // staged from a multiple of 4 (floor for negatives)
    const bool staged = bx0 + bw - bxa <= win.cols && bh <= win.rows;
    if (staged) {
      // window columns [bxa, bx0 + bw) (bxa = bx0 rounded down to 4) of rows
      // by0 .. by0 + bh - 1, four pixels per item: one 4- or 12-byte load,
      // one 16-byte LDS store per channel plane
      const int32_t ngrp = (bx0 + bw - bxa + 3) >> 2;
      for (int i = tid; i < bh * ngrp; i += kLT) {
        const int r = i / ngrp, gq = i - r * ngrp;
        const int32_t y = by0 + r, x = bxa + 4 * gq;
        const bool rowok = y >= 0 && y < P.H;
        const uint8_t* row = sbase + (int64_t)(rowok ? y : 0) * P.pitch;
        const bool full = rowok && x >= 0 && x + 4 <= P.W;
        if constexpr (C == 3) {
          uint4 q;
          if (full) {
            const uint32_t* p3 = reinterpret_cast<const uint32_t*>(row + 3 * (int64_t)x);
            const uint32_t w0 = p3[0], w1 = p3[1], w2 = p3[2];  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
            q = make_uint4(w0, __builtin_amdgcn_alignbyte(w1, w0, 3),
                           __builtin_amdgcn_alignbyte(w2, w1, 2), w2 >> 8);
          } else {
            // window edge: pixels outside the image are white (get_pixel)
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const int32_t xx = x + j;
              const uint8_t* px = row + 3 * (int64_t)xx;
              v[j] = rowok && xx >= 0 && xx < P.W ? (uint32_t)px[0] | (uint32_t)px[1] << 8 | (uint32_t)px[2] << 16
                                                   : 0xFFFFFFu;
            }
            q = make_uint4(v[0], v[1], v[2], v[3]);
          }
          *reinterpret_cast<uint4*>(lwu + r * win.stride + 4 * gq) = q;
        } else {
          float4 q;
          if (full) {
            const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + x);
            q = make_float4(ubyte_f<0>(w0), ubyte_f<1>(w0), ubyte_f<2>(w0), ubyte_f<3>(w0));
          } else {
            float v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const int32_t xx = x + j;
              v[j] = rowok && xx >= 0 && xx < P.W ? (float)row[xx] : 255.0f;
            }
            q = make_float4(v[0], v[1], v[2], v[3]);
          }
          *reinterpret_cast<float4*>(lw + r * win.stride + 4 * gq) = q;
        }
      }
    }
    __syncthreads();
    // 3. the in-mask pixels of this wave's rows
    const int32_t x = tx0 + lane;
    const int32_t u = x - a.mask.x0;
    const bool colin = x < P.W && u >= 0 && u < sw;
    const float cu = u - tcx;
    const float ax = scx + cu * a.cosval, bs = cu * a.sinval;
    // source coordinates of the pixel in tile row r (deskew.c:264-268)
    auto coords = [&](int r, float* cx, float* cy) -> bool {
      const int32_t y = ty0 + r, v = y - a.mask.y0;
      const float cv = v - tcy;
      *cx = ax + cv * a.sinval;          // scx + (u-tcx) cos + (v-tcy) sin
      *cy = (scy + cv * a.cosval) - bs;  // scy + (v-tcy) cos - (u-tcx) sin
      return colin && y < P.H && v >= 0 && v < sh;
    };
    if (!staged) {
      // window too large for LDS (angles far beyond the scan range): taps
      // from the frame
      const Src<FMT> S{sbase, P.pitch, P.W, P.H};
#pragma unroll 1
      for (int k = 0; k < kLRows; k++) {
        const int r = wv * kLRows + k;
        float cx, cy;
        if (!coords(r, &cx, &cy)) continue;
        const Px p = interp_bilinear(S, cx, cy);
        uint8_t* o = obuf + r * kRowB + lane * C;
        o[0] = p.r;
        if (C == 3) {
          o[1] = p.g;
          o[2] = p.b;
        }
      }
    } else {
      // linear_scale as one packed multiply of (1 - f, f) by the tap pair
      // (a, b) -- the pair one ds_read2_b32 returns -- then the add and the
      // truncation: every rounding of (1.0f - f) * a + f * b kept
#pragma unroll 2
      for (int k = 0; k < kLRows; k++) {
        const int r = wv * kLRows + k;
        float cx, cy;
        if (!coords(r, &cx, &cy)) continue;
        // interp_bilinear (interpolate.c:77-118): x2 = ceil = x1 + 1 unless
        // the coordinate is integral; outside the image or with an integral
        // coordinate the result is the pixel (x1, y1) -- the one-axis cases
        // use the other axis' zero fraction
        const float fx1 = floorf(cx), fy1 = floorf(cy);
        const float fx = cx - fx1, fy = cy - fy1;
        const int32_t x1 = (int32_t)fx1, y1 = (int32_t)fy1;
        const bool plain = fx == 0.0f || fy == 0.0f || x1 + 1 < 0 || x1 + 1 > P.W - 1 ||
                           y1 + 1 < 0 || y1 + 1 > P.H - 1;
        const lf2 FX{1.0f - fx, fx}, FY{1.0f - fy, fy};
        // (x1, y1) .. (x1 + 1, y1 + 1) lie in the window
        const int32_t i11 = __mul24(y1 - by0, win.stride) + (x1 - bxa);
        uint8_t* o = obuf + r * kRowB + lane * C;
        if constexpr (C == 3) {
          // one ds_read2_b32 per tap row: pixels (x1, x2) as rgb words
          const uint32_t* q = lwu + i11;
          const uint32_t w11 = q[0], w21 = q[1], w12 = q[win.stride], w22 = q[win.stride + 1];
          // red and green as packed pairs across the channels, blue as the
          // (x1, x2) pair; branch-free, the plain case selected at the end
          const lf2 FX0{FX.x, FX.x}, FX1{FX.y, FX.y}, FY0{FY.x, FY.x}, FY1{FY.y, FY.y};
          const lf2 rg11{ubyte_f<0>(w11), ubyte_f<1>(w11)}, rg21{ubyte_f<0>(w21), ubyte_f<1>(w21)};
          const lf2 rg12{ubyte_f<0>(w12), ubyte_f<1>(w12)}, rg22{ubyte_f<0>(w22), ubyte_f<1>(w22)};
          const lf2 st = FX0 * rg11 + FX1 * rg21, sb = FX0 * rg12 + FX1 * rg22;
          const lf2 ht{__builtin_truncf(st.x), __builtin_truncf(st.y)};
          const lf2 hb{__builtin_truncf(sb.x), __builtin_truncf(sb.y)};
          const lf2 sv = FY0 * ht + FY1 * hb;
          const lf2 tb = FX * lf2{ubyte_f<2>(w11), ubyte_f<2>(w21)};
          const lf2 bb = FX * lf2{ubyte_f<2>(w12), ubyte_f<2>(w22)};
          const lf2 hbl{__builtin_truncf(tb.x + tb.y), __builtin_truncf(bb.x + bb.y)};
          const lf2 fb = FY * hbl;
          // integral values: the byte conversion's rounding is exact
          uint32_t px = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_truncf(sv.x), 0, 0u);
          px = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_truncf(sv.y), 1, px);
          px = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_truncf(fb.x + fb.y), 2, px);
          if (plain) px = w11;
          o[0] = (uint8_t)px;
          o[1] = (uint8_t)(px >> 8);
          o[2] = (uint8_t)(px >> 16);
        } else {
          const float* q = lw + i11;
          const lf2 top{q[0], q[1]}, bot{q[win.stride], q[win.stride + 1]};
          const lf2 t = FX * top, b = FX * bot;
          const lf2 h{__builtin_truncf(t.x + t.y), __builtin_truncf(b.x + b.y)};
          const lf2 f = FY * h;
          o[0] = (uint8_t)(uint32_t)(plain ? top.x : __builtin_truncf(f.x + f.y));
        }
      }
    }
    __syncthreads();  // the next mask restages the window
  }
  // 4. the tile's rows out of LDS, 16 bytes per lane
  {
    constexpr int NV = kRowB / 16;
    for (int i = tid; i < th * NV; i += kLT) {
      const int r = i / NV, j = i - r * NV;
      if (16 * j >= rowb) continue;
      uint8_t* dp = dbase + (int64_t)(ty0 + r) * P.pitch + xb0 + 16 * j;
      const uint4 v = *reinterpret_cast<const uint4*>(obuf + r * kRowB + 16 * j);
      if (vec_ok(j) && 16 * (j + 1) <= rowb) {
        *reinterpret_cast<uint4*>(dp) = v;
      } else {
        const uint32_t wv4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; k++)
          if (16 * j + k < rowb) dp[k] = (uint8_t)(wv4[k >> 2] >> (8 * (k & 3)));
      }
    }
  }
}

LinWindow lin_window(float max_abs_angle) {
  const float a = fminf(fabsf(max_abs_angle), 1.5707964f);
  const float sn = sinf(a), cs = cosf(a);
  LinWindow w;
  // (n-1) cos + (m-1) sin pixel centres, + 1 for ceil, + 2 for the floor of
  // the bounds and the rounding of the corner products; columns + 3 for the
  // start rounded down to a multiple of 4 and up to whole groups of 4
  w.cols = ((int32_t)ceilf((kLW - 1) * cs + (kLH - 1) * sn) + 4 + 3 + 3) & ~3;
  w.rows = (int32_t)ceilf((kLH - 1) * cs + (kLW - 1) * sn) + 4;
  w.stride = w.cols;
  return w;
}

size_t lin_lds_bytes(const LinWindow& w, int fmt) {
  const int C = fmt == F_RGB24 ? 3 : 1;
  return sizeof(float) * (size_t)w.rows * w.stride + (size_t)kLH * kLW * C;
}

bool launch_rotate_linear(const PlaneRef& src, const PlaneRef& dst, const RotateArgs* args,
                          int nmask, int64_t mstride, const int32_t* indep, int count,
                          hipStream_t st, float max_abs_angle) {
  if (src.P.fmt != F_GRAY8 && src.P.fmt != F_RGB24) return false;
  const LinWindow w = lin_window(max_abs_angle);
  const size_t lds = lin_lds_bytes(w, src.P.fmt);
  if (lds > 64 * 1024) return false;
  const dim3 grid((src.P.W + kLW - 1) / kLW, (src.P.H + kLH - 1) / kLH, count);
  const uint32_t mgxy = div_magic(grid.x * grid.y), mgx = div_magic(grid.x);
  if (src.P.fmt == F_RGB24) {
    allow_dynamic_lds((const void*)k_rotate_lin<F_RGB24>, lds);
    hipLaunchKernelGGL(k_rotate_lin<F_RGB24>, grid, dim3(kLT), lds, st, src, dst, args, nmask,
                       mstride, indep, w, mgxy, mgx);
  } else {
    allow_dynamic_lds((const void*)k_rotate_lin<F_GRAY8>, lds);
    hipLaunchKernelGGL(k_rotate_lin<F_GRAY8>, grid, dim3(kLT), lds, st, src, dst, args, nmask,
                       mstride, indep, w, mgxy, mgx);
  }
  return true;
}

}  // namespace uph
