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

// Flag rows of groups up to 64 blocks wide go through LDS: a ring of four
// stripe rows (the stripes above, at and below the one being decoded, and
// the next one arriving), each row the 64 lanes' words of Wg + 2 columns.
// 0: flags straight from the slot (measured faster: 6 waves a SIMD hide the
// slot's latency better than the ring's LDS lets one wave a SIMD hide
// nothing; 209 vs 293 ms per 32-page launch)
#ifndef UPH_T1_RING
#define UPH_T1_RING 0
#endif
constexpr int kRingCols = UPH_T1_RING ? 66 : 0;
constexpr int kRingRow = kRingCols * 64;  // uint16 words

// one flag row between the scratch slot (global) and a ring row (LDS), as
// 16-byte chunks across the lanes (the layouts are the same)
__device__ __forceinline__ void t1_row_load(const uint16_t* g, int ws, uint4 (&r)[9]) {
  const int n16 = ws * 8;  // 16-byte chunks in the row (ws * 64 words)
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int ch = i * 64 + threadIdx.x;
    if (ch < n16) r[i] = reinterpret_cast<const uint4*>(g)[ch];
  }
}
__device__ __forceinline__ void t1_row_put(uint16_t* l, int ws, const uint4 (&r)[9]) {
  const int n16 = ws * 8;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int ch = i * 64 + threadIdx.x;
    if (ch < n16) reinterpret_cast<uint4*>(l)[ch] = r[i];
  }
}
__device__ __forceinline__ void t1_row_store(uint16_t* g, int ws, const uint16_t* l) {
  const int n16 = ws * 8;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int ch = i * 64 + threadIdx.x;
    if (ch < n16) reinterpret_cast<uint4*>(g)[ch] = reinterpret_cast<const uint4*>(l)[ch];
  }
}

// t1_decode_lane with the flag rows in the LDS ring (groups with Wg <= 64):
// each pass loads the first three rows, then per stripe prefetches the row
// two below into registers, decodes the stripe from LDS, writes the stripe's
// row back to the slot and puts the prefetched row in the freed ring row.
// The rows cross lanes on their way (16-byte chunks), so the slot's writes
// and the next pass's reads are ordered by the workgroup (one wave) barrier.
__device__ __attribute__((noinline)) void t1_decode_ring(T1Lane<64>& L, bool active, const uint8_t* data, int numbps,
                               int npasses, int Sg, int maxpasses, uint16_t* ring,
                               uint16_t* gfl) {
  const int lane = threadIdx.x;
  const int WS = L.WS;
  for (int i = lane; i < (Sg + 2) * WS * 8; i += 64) reinterpret_cast<uint4*>(gfl)[i] = make_uint4(0, 0, 0, 0);
  L.pm = 1 << 30;
  if (active) {
    L.reset_contexts();
    L.mq_init(data);
  }
  __syncthreads();
  for (int k = 0; k < maxpasses; k++) {
    int type, bpno;
    t1_pass(k, numbps, &type, &bpno);
    const bool on = active && k < npasses && bpno >= 1;
    if (__ballot(on) == 0) continue;
    if (on && type == 1) L.pm = bpno;
    {
      uint4 r[9];
      for (int R = 0; R < 3 && R <= Sg + 1; R++) {
        t1_row_load(gfl + (int64_t)R * WS * 64, WS, r);
        t1_row_put(ring + R * kRingRow, WS, r);
      }
    }
    for (int s = 0; s < Sg; s++) {
      const int R = s + 1;
      uint4 pre[9];
      const bool more = R + 2 <= Sg + 1;
      if (more) t1_row_load(gfl + (int64_t)(R + 2) * WS * 64, WS, pre);
      const uint16_t* U = ring + ((R - 1) & 3) * kRingRow + lane;
      uint16_t* M = ring + (R & 3) * kRingRow + lane;
      const uint16_t* D = ring + ((R + 1) & 3) * kRingRow + lane;
      uint32_t Ul = 0, Ml = 0, Dl = 0;
      uint32_t Uc = U[64], Mc = M[64], Dc = D[64];
      uint32_t Ur = U[128], Mr = M[128], Dr = D[128];
      const bool srow = on && 4 * s < L.h;
      for (int col = 0; col < L.Wg; col++) {
        uint32_t Un = 0, Mn = 0, Dn = 0;
        if (col + 2 <= L.Wg) {
          Un = U[(col + 3) * 64];
          Mn = M[(col + 3) * 64];
          Dn = D[(col + 3) * 64];
        }
        if (srow && col < L.w) {
          L.column(type, bpno, s, col, Ul, Ml, Dl, Uc, &Mc, Dc, Ur, Mr, Dr);
          M[(col + 1) * 64] = (uint16_t)Mc;
        }
        Ul = Uc;
        Uc = Ur;
        Ur = Un;
        Ml = Mc;
        Mc = Mr;
        Mr = Mn;
        Dl = Dc;
        Dc = Dr;
        Dr = Dn;
      }
      __builtin_amdgcn_wave_barrier();  // this wave's LDS writes land in order before its reads
      t1_row_store(gfl + (int64_t)R * WS * 64, WS, ring + (R & 3) * kRingRow);
      if (more) t1_row_put(ring + ((R + 2) & 3) * kRingRow, WS, pre);
    }
    __syncthreads();  // the rows written back before the next pass reads them
  }
}

// The encoder's passes with the flag rows in the LDS ring (as
// t1_decode_ring); the magnitudes' stripe-column words from the slot,
// prefetched a column ahead.
__device__ __attribute__((noinline)) int32_t t1_encode_ring(T1EncLane<64>& L, bool active, int nb, int Sg, int maxpasses,
                                  uint16_t* ring, uint16_t* gfl) {
  const int lane = threadIdx.x;
  const int WS = L.WS;
  if (active) {
    L.reset_contexts();
    L.init();
  }
  __syncthreads();  // the slot's preset flags (other lanes' chunks below)
  for (int k = 0; k < maxpasses; k++) {
    int type, p;
    t1_pass(k, nb - 1, &type, &p);
    const bool on = active && k < 3 * nb - 2;
    if (__ballot(on) == 0) continue;
    {
      uint4 r[9];
      for (int R = 0; R < 3 && R <= Sg + 1; R++) {
        t1_row_load(gfl + (int64_t)R * WS * 64, WS, r);
        t1_row_put(ring + R * kRingRow, WS, r);
      }
    }
    for (int s = 0; s < Sg; s++) {
      const int R = s + 1;
      uint4 pre[9];
      const bool more = R + 2 <= Sg + 1;
      if (more) t1_row_load(gfl + (int64_t)(R + 2) * WS * 64, WS, pre);
      const uint16_t* U = ring + ((R - 1) & 3) * kRingRow + lane;
      uint16_t* M = ring + (R & 3) * kRingRow + lane;
      const uint16_t* D = ring + ((R + 1) & 3) * kRingRow + lane;
      uint32_t Ul = 0, Ml = 0, Dl = 0;
      uint32_t Uc = U[64], Mc = M[64], Dc = D[64];
      uint32_t Ur = U[128], Mr = M[128], Dr = D[128];
      const bool srow = on && 4 * s < L.h;
      uint64_t m4 = L.M4(s, 0), m4n = 0;
      for (int col = 0; col < L.Wg; col++) {
        uint32_t Un = 0, Mn = 0, Dn = 0;
        if (col + 2 <= L.Wg) {
          Un = U[(col + 3) * 64];
          Mn = M[(col + 3) * 64];
          Dn = D[(col + 3) * 64];
        }
        if (col + 1 < L.Wg) m4n = L.M4(s, col + 1);
        if (srow && col < L.w) {
          L.column(type, p, s, m4, Ul, Ml, Dl, Uc, &Mc, Dc, Ur, Mr, Dr);
          M[(col + 1) * 64] = (uint16_t)Mc;
        }
        m4 = m4n;
        Ul = Uc;
        Uc = Ur;
        Ur = Un;
        Ml = Mc;
        Mc = Mr;
        Mr = Mn;
        Dl = Dc;
        Dc = Dr;
        Dr = Dn;
      }
      __builtin_amdgcn_wave_barrier();
      t1_row_store(gfl + (int64_t)R * WS * 64, WS, ring + (R & 3) * kRingRow);
      if (more) t1_row_put(ring + ((R + 2) & 3) * kRingRow, WS, pre);
    }
    __syncthreads();
  }
  return active ? L.flush() : 0;
}

// Register budgets (waves a SIMD; 0: the compiler's choice, 98-105 VGPRs =
// 4 waves): several code-block launches share the SIMDs, and each lane's
// flag and context traffic is latency, so more resident waves pay even with
// a few spilled registers (JP2 runner A/B: 4 -> 6 waves 847 -> 965-975
// pages/s; 5 and 7 waves 927, 8 waves spill 124 bytes a lane: 772).  The
// encoder at 6 waves measured no different (jp2_write 133 vs 134 pages/s).
#ifndef UPH_T1_WAVES
#define UPH_T1_WAVES 6
#endif
#ifndef UPH_T1ENC_WAVES
#define UPH_T1ENC_WAVES 0
#endif
#if UPH_T1_WAVES > 0
#define UPH_T1_ATTR __attribute__((amdgpu_waves_per_eu(UPH_T1_WAVES)))
#else
#define UPH_T1_ATTR
#endif
#if UPH_T1ENC_WAVES > 0
#define UPH_T1ENC_ATTR __attribute__((amdgpu_waves_per_eu(UPH_T1ENC_WAVES)))
#else
#define UPH_T1ENC_ATTR
#endif

// EBCOT code-block encode, a lane per block: the block's magnitudes and
// preset signs into the slot (lane-minor), its plane count, then every pass
// (flags through the LDS ring when the group is at most 64 wide); the
// codeword into the job's output region.
__global__ void __launch_bounds__(64) UPH_T1ENC_ATTR k_j2k_t1enc(const T1EncJob* jobs, int njobs,
                                                  const uint32_t* coef, uint8_t* dout,
                                                  uint32_t* dlen, uint8_t* dnb, uint8_t* scr,
                                                  int64_t slot_bytes, int64_t mg_off) {
  __shared__ MqState qe[47];
  __shared__ uint8_t zct[kZcTable];
  __shared__ uint8_t cxs[kNumCtx * 64];
  __shared__ __attribute__((aligned(16))) uint16_t ring[UPH_T1_RING ? 4 * kRingRow : 8];
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
    T1EncJob job{};
    if (active) job = jobs[j];
    const int Wg = wave_max(job.w), Hg = wave_max(job.h);
    const int Sg = (Hg + 3) >> 2, WS = Wg + 2;
    uint16_t* fl = reinterpret_cast<uint16_t*>(slot) + lane;
    uint64_t* mg = reinterpret_cast<uint64_t*>(slot + mg_off) + lane;
    // magnitudes and signs, lane-minor; the plane count
    uint32_t mor = 0;
    for (int R = 0; R < Sg + 2; R++)
      for (int col = -1; col <= Wg; col++) {
        const int s = R - 1;
        uint32_t f = 0;
        uint64_t m4 = 0;
        if (active && s >= 0 && s < Sg && col >= 0 && col < job.w) {
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int y = 4 * s + r;
            if (y < job.h) {
              const int32_t v = (int32_t)coef[job.in + (int64_t)y * job.stride + col];
              const uint32_t a = (uint32_t)(v < 0 ? -v : v);
              mor |= a;
              m4 |= (uint64_t)(a & 0xFFFFu) << (16 * r);
              if (v < 0) f |= 2u << (4 * r);
            }
          }
        }
        fl[(int64_t)(R * WS + col + 1) * 64] = (uint16_t)f;
        if (s >= 0 && s < Sg && col >= 0 && col < Wg) mg[(int64_t)(s * Wg + col) * 64] = m4;
      }
    int nb = mor ? 32 - __builtin_clz(mor) : 0;
    if (nb > 16) {  // beyond the 16-bit magnitude words (not from 8-bit samples): refused
      if (active) dnb[j] = 0xFF;
      nb = 0;
    }
    const int P = wave_max(nb > 0 ? 3 * nb - 2 : 0);
    T1EncLane<64> L;
    L.WS = WS;
    L.Wg = Wg;
    L.fl = fl;
    L.mg = mg;
    L.cx = cxs + lane;
    L.qe = qe;
    L.zct = zct;
    L.w = job.w;
    L.h = job.h;
    L.orient = job.orient;
    L.out = dout + job.out;
    L.cap = (int32_t)t1_enc_cap(job.w, job.h);
    L.over = false;  // (init() runs only for blocks with planes)
    int32_t n;
    if (WS <= kRingCols)
      n = t1_encode_ring(L, active && nb > 0, nb, Sg, P, ring, reinterpret_cast<uint16_t*>(slot));
    else
      n = t1_encode_lane(L, active && nb > 0, nb, Sg, P, [](bool b) { return __ballot(b) != 0; });
    if (active) {
      dlen[j] = L.over ? 0u : (uint32_t)n;
      if (mor < 0x10000u) dnb[j] = L.over ? 0xFE : (uint8_t)nb;  // > 16: refused by the host
    }
    __syncthreads();  // the slot is rewritten by the next group
  }
}

// exclusive prefix sum of the codeword lengths (one workgroup), total at
// [n]; with `base`, the sums start at *base (read before off[0] is written:
// a chunk's sub-batches chain through it)
__global__ void __launch_bounds__(1024) k_j2k_scan(const uint32_t* len, uint32_t* off, int n,
                                                  const uint32_t* base) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = base ? *base : 0u;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + threadIdx.x;
    const uint32_t v = i < n ? len[i] : 0u;
    uint32_t incl = v;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = (uint32_t)__shfl_up((int)incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = carry;
    for (int k = 0; k < wv; k++) before += wsum[k];
    if (i < n) off[i] = before + incl - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) off[n] = carry;
}

// each job's codeword to its packed offset, a wave a job; past `cap` bytes
// of packed output the job is dropped and *err set
__global__ void __launch_bounds__(256) k_j2k_gather(const T1EncJob* jobs, int njobs,
                                                    const uint8_t* dout, const uint32_t* len,
                                                    const uint32_t* off, uint8_t* packed,
                                                    uint64_t cap, int32_t* err) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= njobs) return;
  if ((uint64_t)off[j] + len[j] > cap) {
    if ((threadIdx.x & 63) == 0 && err) atomicOr(err, 1);
    return;
  }
  const uint8_t* s = dout + jobs[j].out;
  uint8_t* d = packed + off[j];
  for (uint32_t i = threadIdx.x & 63; i < len[j]; i += 64) d[i] = s[i];
}

// EBCOT code-block decode, a lane per block (j2k_t1_lane.h): the MQ tables
// and the context bytes in LDS, flags in the block's scratch slot laid out
// lane-minor (coalesced; through the LDS ring for groups up to 64 wide),
// magnitude bits there too, the decoded block into the coefficients.
__global__ void __launch_bounds__(64) UPH_T1_ATTR k_j2k_t1(const T1Job* jobs, int njobs, const uint8_t* data,
                                               uint32_t* coef, uint8_t* scr, int64_t slot_bytes,
                                               int64_t val_off) {
  __shared__ MqState qe[47];
  __shared__ uint8_t zct[kZcTable];
  __shared__ uint8_t cxs[kNumCtx * 64];
  __shared__ __attribute__((aligned(16))) uint16_t ring[UPH_T1_RING ? 4 * kRingRow : 8];
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
    if (Wg + 2 <= kRingCols)
      t1_decode_ring(L, active, data + job.data, job.numbps, job.npasses, (Hg + 3) >> 2, P, ring,
                     reinterpret_cast<uint16_t*>(slot));
    else
      t1_decode_lane(L, active, data + job.data, job.numbps, job.npasses, (Hg + 3) >> 2, P,
                     [](bool b) { return __ballot(b) != 0; });
    __syncthreads();  // flags written back (other lanes' chunks) before the store reads them
    t1_store_lane(L, active, job, coef, Hg);
  }
}

}  // namespace

size_t t1enc_slot_bytes(int maxw, int maxh) {
  const size_t flags = (((size_t)((maxh + 3) / 4 + 2) * (size_t)(maxw + 2) * 64 * 2) + 255) & ~(size_t)255;
  return flags + (size_t)((maxh + 3) / 4) * (size_t)maxw * 64 * 8;
}

bool t1enc_launch(const T1EncJob* djobs, int njobs, const uint32_t* dcoef, uint8_t* dout,
                  uint32_t* dlen, uint8_t* dnb, void* dscr, int nslots, int maxw, int maxh,
                  hipStream_t st) {
  if (njobs <= 0) return true;
  const int64_t slot = (int64_t)t1enc_slot_bytes(maxw, maxh);
  const int64_t mg_off =
      (int64_t)((((size_t)((maxh + 3) / 4 + 2) * (size_t)(maxw + 2) * 64 * 2) + 255) & ~(size_t)255);
  hipLaunchKernelGGL(k_j2k_t1enc, dim3((unsigned)nslots), dim3(64), 0, st, djobs, njobs, dcoef, dout,
                     dlen, dnb, (uint8_t*)dscr, slot, mg_off);
  return UPH_HIP(hipGetLastError());
}

bool t1enc_pack(const T1EncJob* djobs, int njobs, const uint8_t* dout, const uint32_t* dlen,
                uint32_t* doff, uint8_t* dpacked, uint64_t cap, int32_t* derr, bool chained,
                hipStream_t st) {
  if (njobs <= 0) return true;
  hipLaunchKernelGGL(k_j2k_scan, dim3(1), dim3(1024), 0, st, dlen, doff, njobs,
                     chained ? (const uint32_t*)doff : (const uint32_t*)nullptr);
  hipLaunchKernelGGL(k_j2k_gather, dim3((unsigned)((njobs + 3) / 4)), dim3(256), 0, st, djobs, njobs,
                     dout, dlen, doff, dpacked, cap, derr);
  return UPH_HIP(hipGetLastError());
}

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
                   void* vtmp, hipStream_t st) {
  const Tile& t = img.tiles[0];
  const int w = t.x1 - t.x0, h = t.y1 - t.y0;
  int32_t* tmp = (int32_t*)vtmp;
  if (!tmp) return fail("jp2 encode: no line buffer");
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
