// kernels_j2k.hip — the device half of JPEG 2000 (j2k.h): inverse wavelet
// transforms per resolution level (rows, then columns, as OpenJPEG's
// dwt.c and the standard's 2D_SR), the inverse component transform, the DC
// level shift and the store into the destination image; for the lossless
// encoder the DC shift, the forward RCT and the forward 5/3 transform
// (columns, then rows, per level).  A thread per output pair of a line: the
// lifting recomputed over a small window of the line (j2k_dwt.h), each pass
// from one buffer into the other (plane and tmp, the same row stride), the
// column passes' threads along the rows (coalesced).
#include <algorithm>
#include <type_traits>

#include "j2k.h"
#include "j2k_dwt.h"
#include "j2k_t1_lane.h"
#include "runtime.h"

namespace uph {
namespace j2k {

namespace {

// Inverse wavelet of one level, a thread per output pair (j2k_dwt.h
// idwt_pair): rows of the plane (Mallat in x) into tmp in natural order, then
// columns of tmp (Mallat in y) back into the plane; a column pass's threads
// span 64 columns, so every load and store of a row segment is coalesced.
template <class T, int CAS>
__global__ void __launch_bounds__(256) k_j2k_irow(const T* __restrict__ src, T* __restrict__ dst,
                                                  int stride, int rw, int rh) {
  const int y = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (2 * t >= rw) return;
  const T* line = src + (int64_t)y * stride;
  T o0, o1;
  idwt_pair<T, CAS>(line, 1, rw, t, &o0, &o1);
  T* d = dst + (int64_t)y * stride + 2 * t;
  d[0] = o0;
  if (2 * t + 1 < rw) d[1] = o1;
}
template <class T, int CAS>
__global__ void __launch_bounds__(256) k_j2k_icol(const T* __restrict__ src, T* __restrict__ dst,
                                                  int stride, int rw, int rh) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int t = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= rw || 2 * t >= rh) return;
  T o0, o1;
  idwt_pair<T, CAS>(src + x, stride, rh, t, &o0, &o1);
  dst[(int64_t)(2 * t) * stride + x] = o0;
  if (2 * t + 1 < rh) dst[(int64_t)(2 * t + 1) * stride + x] = o1;
}

// one tile into the image: inverse MCT, DC shift, clamp, store
template <bool REV>
__global__ void __launch_bounds__(256) k_j2k_out(const uint32_t* coef, Tile t, int ncomp,
                                                 int32_t ox, int32_t oy, uint8_t* dst,
                                                 int64_t pitch) {
  const int w = t.x1 - t.x0, h = t.y1 - t.y0;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)w * h) return;
  const int x = (int)(i % w), y = (int)(i / w);
  uint8_t* d = dst + (int64_t)(t.y0 + y - oy) * pitch;
  const int X = t.x0 + x - ox;
  auto at = [&](int c) { return coef[t.tc[c].off + (int64_t)y * t.tc[c].stride + x]; };
  if (ncomp == 1) {
    if (REV) d[X] = clamp8((int32_t)at(0) + 128);
    else d[X] = clamp8(round_half_even(__uint_as_float(at(0))) + 128);
    return;
  }
  uint8_t r, g, b;
  if (REV) {
    const int32_t y0 = (int32_t)at(0), y1 = (int32_t)at(1), y2 = (int32_t)at(2);
    if (t.mct) {
      rct_inverse(y0, y1, y2, &r, &g, &b);
    } else {
      r = clamp8(y0 + 128);
      g = clamp8(y1 + 128);
      b = clamp8(y2 + 128);
    }
  } else {
    const float y0 = __uint_as_float(at(0)), y1 = __uint_as_float(at(1)), y2 = __uint_as_float(at(2));
    if (t.mct) {
      ict_inverse(y0, y1, y2, &r, &g, &b);
    } else {
      r = clamp8(round_half_even(y0) + 128);
      g = clamp8(round_half_even(y1) + 128);
      b = clamp8(round_half_even(y2) + 128);
    }
  }
  d[3 * X] = r;
  d[3 * X + 1] = g;
  d[3 * X + 2] = b;
}

// encoder: image -> DC-shifted (and RCT-transformed) integer planes
__global__ void __launch_bounds__(256) k_j2k_in(const uint8_t* src, int64_t pitch, int w, int h,
                                                int ncomp, uint32_t* coef) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)w * h) return;
  const int x = (int)(i % w), y = (int)(i / w);
  const uint8_t* s = src + (int64_t)y * pitch;
  const int64_t n = (int64_t)w * h;
  if (ncomp == 1) {
    coef[i] = (uint32_t)((int32_t)s[x] - 128);
    return;
  }
  const int32_t R = (int32_t)s[3 * x] - 128, G = (int32_t)s[3 * x + 1] - 128,
                B = (int32_t)s[3 * x + 2] - 128;
  coef[i] = (uint32_t)((R + 2 * G + B) >> 2);  // RCT (G.2.1)
  coef[n + i] = (uint32_t)(B - G);
  coef[2 * n + i] = (uint32_t)(R - G);
}

// Forward 5/3 of one level (encoder), a thread per input pair: columns of
// the plane (natural) into tmp (Mallat in y), then rows of tmp (natural in
// x) back into the plane (Mallat in x).
template <int CAS>
__global__ void __launch_bounds__(256) k_j2k_fcol(const int32_t* __restrict__ src,
                                                  int32_t* __restrict__ dst, int stride, int rw,
                                                  int rh) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int t = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= rw || 2 * t >= rh) return;
  int32_t o0, o1;
  fdwt53_pair<CAS>(src + x, stride, rh, t, &o0, &o1);
  dst[(int64_t)mallat_index(2 * t, rh, CAS) * stride + x] = o0;
  if (2 * t + 1 < rh) dst[(int64_t)mallat_index(2 * t + 1, rh, CAS) * stride + x] = o1;
}
template <int CAS>
__global__ void __launch_bounds__(256) k_j2k_frow(const int32_t* __restrict__ src,
                                                  int32_t* __restrict__ dst, int stride, int rw,
                                                  int rh) {
  const int y = blockIdx.y;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (2 * t >= rw) return;
  int32_t o0, o1;
  fdwt53_pair<CAS>(src + (int64_t)y * stride, 1, rw, t, &o0, &o1);
  int32_t* d = dst + (int64_t)y * stride;
  d[mallat_index(2 * t, rw, CAS)] = o0;
  if (2 * t + 1 < rw) d[mallat_index(2 * t + 1, rw, CAS)] = o1;
}

unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// EBCOT code-block decode, a lane per block (j2k_t1_lane.h): the MQ tables
// and the context bytes in LDS, flags and values in the block's scratch slot
// laid out lane-minor (coalesced), the decoded block into the coefficients.
__global__ void __launch_bounds__(64) k_j2k_t1(const T1Job* jobs, int njobs, const uint8_t* data,
                                               uint32_t* coef, uint8_t* scr, int64_t slot_bytes,
                                               int64_t val_off) {
  __shared__ MqState qe[47];
  __shared__ uint8_t zct[kZcTable];
  __shared__ uint8_t cxs[kNumCtx * 64];
  const int lane = threadIdx.x;
  if (lane < 47) qe[lane] = kMq[lane];
  for (int i = lane; i < kZcTable; i += 64) {
    const int r = i % 45;
    zct[i] = (uint8_t)zc_ctx(i / 45, r / 15, (r / 5) % 3, r % 5);
  }
  __syncthreads();
  const int ngroups = (njobs + 63) >> 6;
  uint8_t* slot = scr + (int64_t)blockIdx.x * slot_bytes;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int j = g * 64 + lane;
    const bool active = j < njobs;
    T1Job job{};
    if (active) job = jobs[j];
    const int Wg = wave_max(job.w), Hg = wave_max(job.h), P = wave_max(job.npasses);
    T1Lane<64> L;
    L.WS = Wg + 2;
    L.Wg = Wg;
    L.fl = reinterpret_cast<uint16_t*>(slot) + lane;
    L.val = reinterpret_cast<uint32_t*>(slot + val_off) + lane;
    L.cx = cxs + lane;
    L.qe = qe;
    L.zct = zct;
    L.w = job.w;
    L.h = job.h;
    L.orient = job.orient;
    t1_decode_lane(L, active, data + job.data, job.numbps, job.npasses, (Hg + 3) >> 2, P,
                   [](bool b) { return __ballot(b) != 0; });
    t1_store_lane(L, active, job, coef, Hg);
  }
}

}  // namespace

size_t t1_slot_bytes(int maxw, int maxh) {
  const size_t flags = (((size_t)((maxh + 3) / 4 + 2) * (size_t)(maxw + 2) * 64 * 2) + 255) & ~(size_t)255;
  return flags + (size_t)maxw * (size_t)maxh * 64 * 4;
}

bool t1_launch(const T1Job* djobs, int njobs, const uint8_t* ddata, uint32_t* dcoef, void* dscr,
               int nslots, int maxw, int maxh, hipStream_t st) {
  if (njobs <= 0) return true;
  const int64_t slot = (int64_t)t1_slot_bytes(maxw, maxh);
  const int64_t val_off =
      (int64_t)((((size_t)((maxh + 3) / 4 + 2) * (size_t)(maxw + 2) * 64 * 2) + 255) & ~(size_t)255);
  hipLaunchKernelGGL(k_j2k_t1, dim3((unsigned)nslots), dim3(64), 0, st, djobs, njobs, ddata, dcoef,
                     (uint8_t*)dscr, slot, val_off);
  return UPH_HIP(hipGetLastError());
}

size_t decode_tmp_bytes(const Image& img) {
  int64_t tmp_elems = 1;
  for (const Tile& t : img.tiles)
    tmp_elems = std::max<int64_t>(tmp_elems, (int64_t)(t.x1 - t.x0) * (t.y1 - t.y0));
  return (size_t)tmp_elems * 4;
}

bool decode_launch(const Image& img, uint32_t* dcoef, uint8_t* dst, int64_t pitch, void* vtmp,
                   hipStream_t st) {
  uint32_t* tmp = (uint32_t*)vtmp;
  if (!tmp) return fail("jp2: no line buffer");
  for (const Tile& t : img.tiles) {
    for (int c = 0; c < img.ncomp; c++) {
      const TileComp& tc = t.tc[c];
      for (int r = 1; r <= tc.nlevels; r++) {
        const int rw = tc.rx1[r] - tc.rx0[r], rh = tc.ry1[r] - tc.ry0[r];
        if (rw <= 0 || rh <= 0) continue;
        uint32_t* plane = dcoef + tc.off;
        const dim3 rg((unsigned)((rw + 511) / 512), (unsigned)rh);
        const dim3 cg((unsigned)((rw + 63) / 64), (unsigned)((rh + 7) / 8));
        const int cx = tc.rx0[r] & 1, cy = tc.ry0[r] & 1;
        if (img.reversible) {
          int32_t* pl = (int32_t*)plane;
          int32_t* tp = (int32_t*)tmp;
          if (cx) hipLaunchKernelGGL((k_j2k_irow<int32_t, 1>), rg, dim3(256), 0, st, pl, tp, tc.stride, rw, rh);
          else hipLaunchKernelGGL((k_j2k_irow<int32_t, 0>), rg, dim3(256), 0, st, pl, tp, tc.stride, rw, rh);
          if (cy) hipLaunchKernelGGL((k_j2k_icol<int32_t, 1>), cg, dim3(256), 0, st, tp, pl, tc.stride, rw, rh);
          else hipLaunchKernelGGL((k_j2k_icol<int32_t, 0>), cg, dim3(256), 0, st, tp, pl, tc.stride, rw, rh);
        } else {
          float* pl = (float*)plane;
          float* tp = (float*)tmp;
          if (cx) hipLaunchKernelGGL((k_j2k_irow<float, 1>), rg, dim3(256), 0, st, pl, tp, tc.stride, rw, rh);
          else hipLaunchKernelGGL((k_j2k_irow<float, 0>), rg, dim3(256), 0, st, pl, tp, tc.stride, rw, rh);
          if (cy) hipLaunchKernelGGL((k_j2k_icol<float, 1>), cg, dim3(256), 0, st, tp, pl, tc.stride, rw, rh);
          else hipLaunchKernelGGL((k_j2k_icol<float, 0>), cg, dim3(256), 0, st, tp, pl, tc.stride, rw, rh);
        }
      }
    }
    const int64_t npx = (int64_t)(t.x1 - t.x0) * (t.y1 - t.y0);
    if (img.reversible)
      hipLaunchKernelGGL(k_j2k_out<true>, dim3(blocks(npx)), dim3(256), 0, st, dcoef, t, img.ncomp,
                         img.x0, img.y0, dst, pitch);
    else
      hipLaunchKernelGGL(k_j2k_out<false>, dim3(blocks(npx)), dim3(256), 0, st, dcoef, t, img.ncomp,
                         img.x0, img.y0, dst, pitch);
  }
  return UPH_HIP(hipGetLastError());
}

bool encode_launch(const Image& img, const uint8_t* src, int64_t pitch, uint32_t* dcoef,
                   hipStream_t st) {
  const Tile& t = img.tiles[0];
  const int w = t.x1 - t.x0, h = t.y1 - t.y0;
  int32_t* tmp = (int32_t*)scratch(7, (size_t)w * h * 4);
  if (!tmp) return false;
  hipLaunchKernelGGL(k_j2k_in, dim3(blocks((int64_t)w * h)), dim3(256), 0, st, src, pitch, w, h,
                     img.ncomp, dcoef);
  for (int c = 0; c < img.ncomp; c++) {
    const TileComp& tc = t.tc[c];
    int32_t* plane = (int32_t*)(dcoef + tc.off);
    for (int r = tc.nlevels; r >= 1; r--) {
      const int rw = tc.rx1[r] - tc.rx0[r], rh = tc.ry1[r] - tc.ry0[r];
      if (rw <= 0 || rh <= 0) continue;
      const dim3 rg((unsigned)((rw + 511) / 512), (unsigned)rh);
      const dim3 cg((unsigned)((rw + 63) / 64), (unsigned)((rh + 7) / 8));
      if (tc.ry0[r] & 1) hipLaunchKernelGGL(k_j2k_fcol<1>, cg, dim3(256), 0, st, plane, tmp, tc.stride, rw, rh);
      else hipLaunchKernelGGL(k_j2k_fcol<0>, cg, dim3(256), 0, st, plane, tmp, tc.stride, rw, rh);
      if (tc.rx0[r] & 1) hipLaunchKernelGGL(k_j2k_frow<1>, rg, dim3(256), 0, st, tmp, plane, tc.stride, rw, rh);
      else hipLaunchKernelGGL(k_j2k_frow<0>, rg, dim3(256), 0, st, tmp, plane, tc.stride, rw, rh);
    }
  }
  return UPH_HIP(hipGetLastError());
}

}  // namespace j2k
}  // namespace uph
