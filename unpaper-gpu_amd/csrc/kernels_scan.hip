// kernels_scan.hip — axis reductions and the sequential scans that consume
// them: detect_edge / detect_mask (masks.c:54-209), detect_border_edge /
// detect_border (masks.c:410-488).
//
// The reference evaluates every scan bar independently by re-reading its
// 50 x H pixels (29 % of CPU time).  Here one streaming pass produces the
// per-column (or per-row) sums over the bar's fixed extent; every bar sum is
// then a sum of <= size entries from LDS, and the sequential stopping rule
// becomes a block-wide prefix scan + first-failure search (bit-exact: integer
// sums, the same float expression for the threshold test).
#include <climits>

#include "scan.h"

namespace uph {

constexpr int kRedThreads = 256;

template <int FMT, int MEAS>
__device__ __forceinline__ uint32_t measure(const uint8_t* row, int32_t x, uint8_t thr) {
  Px p = load_px_row<FMT>(row, x);
  if (MEAS == M_GRAY_SUM) return gray_of(p);
  if (MEAS == M_DARK_COUNT) return gray_of(p) <= thr ? 1u : 0u;
  if (MEAS == M_DARKINV_SUM) return dark_of(p);
  return light_of(p);  // M_LIGHT_SUM
}

// axis 0 (column sums): threads own columns, blocks own (column tile, row
// chunk); one atomic per column per block.
template <int FMT, int MEAS>
__global__ void __launch_bounds__(kRedThreads) k_colsum(PlaneRef ref, const AxisArgs* args,
                                                        uint32_t* out, int64_t out_stride,
                                                        int rows_per_block) {
  const int s = blockIdx.z;
  const AxisArgs a = args[s];
  if (!a.active) return;
  const Rect r = a.region;
  const int32_t x = r.x0 + (int32_t)blockIdx.x * kRedThreads + (int32_t)threadIdx.x;
  const int32_t y0 = r.y0 + (int32_t)blockIdx.y * rows_per_block;
  if (r.x1 < r.x0 || x > r.x1 || y0 > r.y1) return;
  const int32_t y1 = imin(r.y1, y0 + rows_per_block - 1);
  const uint8_t* base = plane_ptr(ref, s);
  const int64_t pitch = ref.P.pitch;
  uint32_t acc = 0;
  for (int32_t y = y0; y <= y1; y++)
    acc += measure<FMT, MEAS>(base + (int64_t)y * pitch, x, a.thr);
  if (acc) atomicAdd(out + (int64_t)s * out_stride + x, acc);
}

// axis 1 (row sums): a block per row (grid-strided), block reduction.
template <int FMT, int MEAS>
__global__ void __launch_bounds__(kRedThreads) k_rowsum(PlaneRef ref, const AxisArgs* args,
                                                        uint32_t* out, int64_t out_stride) {
  const int s = blockIdx.z;
  const AxisArgs a = args[s];
  if (!a.active) return;
  const Rect r = a.region;
  if (r.x1 < r.x0) return;
  const uint8_t* base = plane_ptr(ref, s);
  __shared__ uint32_t red[kRedThreads / 64];
  for (int32_t y = r.y0 + (int32_t)blockIdx.x; y <= r.y1; y += gridDim.x) {
    const uint8_t* row = base + (int64_t)y * ref.P.pitch;
    uint32_t acc = 0;
    for (int32_t x = r.x0 + (int32_t)threadIdx.x; x <= r.x1; x += kRedThreads)
      acc += measure<FMT, MEAS>(row, x, a.thr);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t t = 0;
      for (int w = 0; w < kRedThreads / 64; w++) t += red[w];
      out[(int64_t)s * out_stride + y] = t;
    }
    __syncthreads();
  }
}

// axis 0 on a gray plane: a lane owns 4 consecutive columns (one aligned
// dword per row; rows start 256-byte aligned, so it lies in the row's pitch),
// the 4 waves of a block take quarters of the block's rows (8 loads in flight
// per lane) and their sums meet in LDS: one atomic per column per block.
template <int MEAS>
__global__ void __launch_bounds__(256) k_colsum_g(PlaneRef ref, const AxisArgs* args, uint32_t* out,
                                                  int64_t out_stride, int rows_per_block) {
  const int s = blockIdx.z;
  const AxisArgs a = args[s];
  if (!a.active) return;
  const Rect r = a.region;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int32_t vx0 = (r.x0 & ~3) + ((int32_t)blockIdx.x * 64 + lane) * 4;
  const int32_t yb = r.y0 + (int32_t)blockIdx.y * rows_per_block;
  if (r.x1 < r.x0 || yb > r.y1) return;
  const int32_t ye = imin(r.y1, yb + rows_per_block - 1);
  const int32_t q = (rows_per_block + 3) / 4;
  const int32_t y0 = yb + w * q, y1 = imin(ye, y0 + q - 1);
  const bool col_ok = vx0 <= r.x1;
  const uint8_t* base = plane_ptr(ref, s) + (col_ok ? vx0 : (r.x0 & ~3));
  const int64_t pitch = ref.P.pitch;
  // the four columns accumulate as 16-bit lanes of two words (bytes 0/2 and
  // 1/3): a wave sums at most rows_per_block / 4 = 64 rows of <= 255, so no
  // lane overflows; two masks and two adds per dword instead of four of each
  static_assert(256 / 4 * 255 < 65536, "16-bit column lanes");
  const uint32_t kadd = (256u - ((uint32_t)a.thr + 1u)) * 0x00010001u;
  uint32_t a02 = 0, a13 = 0;
  for (int32_t y = y0; y <= y1; y += 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++)  // rows past y1 re-read row y1 and are not summed
      v[k] = *reinterpret_cast<const uint32_t*>(base + (int64_t)imin(y + k, y1) * pitch);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t lo = v[k] & 0x00FF00FFu, hi = (v[k] >> 8) & 0x00FF00FFu;
      if (MEAS == M_DARK_COUNT) {  // byte <= thr: bit 8 of byte + 256 - (thr+1) clear
        lo = 0x00010001u - (((lo + kadd) >> 8) & 0x00010001u);
        hi = 0x00010001u - (((hi + kadd) >> 8) & 0x00010001u);
      }
      if (y + k <= y1) {
        a02 += lo;
        a13 += hi;
      }
    }
  }
  const uint32_t acc[4] = {a02 & 0xFFFFu, a13 & 0xFFFFu, a02 >> 16, a13 >> 16};
  __shared__ uint32_t red[4][64 * 4];
#pragma unroll
  for (int j = 0; j < 4; j++) red[w][lane * 4 + j] = acc[j];
  __syncthreads();
  const int c = threadIdx.x;  // 256 columns of the block
  const int32_t x = (r.x0 & ~3) + (int32_t)blockIdx.x * 256 + c;
  const uint32_t t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  if (x >= r.x0 && x <= r.x1 && t) atomicAdd(out + (int64_t)s * out_stride + x, t);
}

// axis 1 on a gray plane: a row is a segment of L lanes (L = the power of
// two covering its 16-byte vectors, at most 64), so narrow regions (the
// blackfilter's vertical stripe) put several rows in one wave.  Every vector
// is measured four bytes at a time: v_sad_u8 sums four bytes, the dark count
// is the popcount of a SWAR compare; only the two edge vectors of a row are
// masked byte by byte.
template <int MEAS>
__device__ __forceinline__ uint32_t measure_g4(uint32_t x, uint32_t keep, uint32_t kadd,
                                               uint32_t acc) {
  if (MEAS == M_DARK_COUNT) {
    const uint32_t lo = ((x & 0x00FF00FFu) + kadd) & 0x01000100u;
    const uint32_t hi = (((x >> 8) & 0x00FF00FFu) + kadd) & 0x01000100u;
    const uint32_t ge = (lo >> 8) | (hi >> 7);                 // byte >= thr+1, bits 0,1,16,17
    const uint32_t lt = ~(ge | (ge >> 14)) & 0xFu;             // bytes <= thr
    const uint32_t kp = (keep & 1u) | ((keep >> 7) & 2u) | ((keep >> 14) & 4u) | ((keep >> 21) & 8u);
    return acc + __popc(lt & kp);
  }
  return __builtin_amdgcn_sad_u8(x & keep, 0u, acc);
}

// a whole dword inside the region (no byte masks)
template <int MEAS>
__device__ __forceinline__ uint32_t measure_g4_full(uint32_t x, uint32_t kadd, uint32_t acc) {
  if (MEAS == M_DARK_COUNT) {  // 4 - (bytes >= thr+1)
    const uint32_t lo = ((x & 0x00FF00FFu) + kadd) & 0x01000100u;
    const uint32_t hi = (((x >> 8) & 0x00FF00FFu) + kadd) & 0x01000100u;
    return acc + 4u - __popc(lo | (hi << 1));
  }
  return __builtin_amdgcn_sad_u8(x, 0u, acc);
}

template <int MEAS>
__global__ void __launch_bounds__(256) k_rowsum_g(PlaneRef ref, const AxisArgs* args, uint32_t* out,
                                                  int64_t out_stride, int seg_log2) {
  const int s = blockIdx.z;
  const AxisArgs a = args[s];
  if (!a.active) return;
  const Rect r = a.region;
  if (r.x1 < r.x0) return;
  const int L = 1 << seg_log2, sl = threadIdx.x & (L - 1);
  const int32_t y = r.y0 + (int32_t)((blockIdx.x * 256 + threadIdx.x) >> seg_log2);
  const bool live = y <= r.y1;
  const uint8_t* row = plane_ptr(ref, s) + (int64_t)(live ? y : r.y0) * ref.P.pitch;
  const int32_t a0 = r.x0 & ~15, nv = ((r.x1 | 15) - a0 + 1) >> 4;
  const uint32_t kadd = (256u - ((uint32_t)a.thr + 1u)) * 0x00010001u;
  uint32_t acc = 0;
  for (int32_t v0 = 0; v0 < nv; v0 += 4 * L) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t vi = v0 + k * L + sl;
      v[k] = *reinterpret_cast<const uint4*>(row + a0 + 16 * (vi < nv ? vi : 0));
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t vi = v0 + k * L + sl;
      if (vi >= nv || !live) continue;
      const int32_t c = a0 + 16 * vi;
      const uint32_t wd[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int32_t x = c + 4 * j;
        if (x >= r.x0 && x + 3 <= r.x1) {
          acc = measure_g4_full<MEAS>(wd[j], kadd, acc);
        } else {
          uint32_t keep = 0;
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (x + q >= r.x0 && x + q <= r.x1) keep |= 0xFFu << (8 * q);
          acc = measure_g4<MEAS>(wd[j], keep, kadd, acc);
        }
      }
    }
  }
  for (int o = L >> 1; o > 0; o >>= 1) acc += __shfl_down(acc, o, L);
  if (sl == 0 && live) out[(int64_t)s * out_stride + y] = acc;
}

template <int FMT, int MEAS>
static void launch_axis_t(const PlaneRef& ref, const AxisArgs* args, int axis, int32_t span_x,
                          int32_t span_y, uint32_t* out, int64_t out_stride, int count,
                          hipStream_t st) {
  if (span_x <= 0 || span_y <= 0) return;
  if (FMT == F_GRAY8) {
    if (axis == 0) {
      const int rpb = 256;  // k_colsum_g's 16-bit column lanes assume <= 256
      dim3 grid((span_x + 3 + 255) / 256, (span_y + rpb - 1) / rpb, count);
      hipLaunchKernelGGL((k_colsum_g<MEAS>), grid, dim3(256), 0, st, ref, args, out, out_stride,
                         rpb);
    } else {
      // lanes per row: the power of two covering a full-width row's vectors
      // (the regions of one launch differ per sheet only in position)
      const int nv = (span_x + 30) / 16;
      int lg = 0;
      while ((1 << lg) < nv && lg < 6) lg++;
      const int64_t rows_per_block = 256 >> lg;
      dim3 grid((unsigned)((span_y + rows_per_block - 1) / rows_per_block), 1, count);
      hipLaunchKernelGGL((k_rowsum_g<MEAS>), grid, dim3(256), 0, st, ref, args, out, out_stride,
                         lg);
    }
    return;
  }
  if (axis == 0) {
    const int rpb = 64;
    dim3 grid((span_x + kRedThreads - 1) / kRedThreads, (span_y + rpb - 1) / rpb, count);
    hipLaunchKernelGGL((k_colsum<FMT, MEAS>), grid, dim3(kRedThreads), 0, st, ref, args, out,
                       out_stride, rpb);
  } else {
    int gx = span_y > 2048 ? 2048 : span_y;
    hipLaunchKernelGGL((k_rowsum<FMT, MEAS>), dim3(gx, 1, count), dim3(kRedThreads), 0, st, ref,
                       args, out, out_stride);
  }
}

template <int FMT>
static void launch_axis_f(const PlaneRef& ref, const AxisArgs* args, int axis, int meas,
                          int32_t sx, int32_t sy, uint32_t* out, int64_t os, int count,
                          hipStream_t st) {
  switch (meas) {
    case M_GRAY_SUM:
      launch_axis_t<FMT, M_GRAY_SUM>(ref, args, axis, sx, sy, out, os, count, st);
      break;
    case M_DARK_COUNT:
      launch_axis_t<FMT, M_DARK_COUNT>(ref, args, axis, sx, sy, out, os, count, st);
      break;
    case M_DARKINV_SUM:
      launch_axis_t<FMT, M_DARKINV_SUM>(ref, args, axis, sx, sy, out, os, count, st);
      break;
    default:
      launch_axis_t<FMT, M_LIGHT_SUM>(ref, args, axis, sx, sy, out, os, count, st);
      break;
  }
}

void launch_axis_reduce(const PlaneRef& ref, const AxisArgs* args, int axis, int meas,
                        int32_t span_x, int32_t span_y, uint32_t* out, int64_t out_stride,
                        int count, hipStream_t st) {
  // axis 0 accumulates with atomics: the caller zeroes `out` first.
  switch (ref.P.fmt) {
    case F_GRAY8:
      launch_axis_f<F_GRAY8>(ref, args, axis, meas, span_x, span_y, out, out_stride, count, st);
      break;
    case F_Y400A:
      launch_axis_f<F_Y400A>(ref, args, axis, meas, span_x, span_y, out, out_stride, count, st);
      break;
    default:
      launch_axis_f<F_RGB24>(ref, args, axis, meas, span_x, span_y, out, out_stride, count, st);
      break;
  }
}

// Block-wide inclusive prefix sum of `v` (256 threads = 4 waves) plus a carry.
__device__ __forceinline__ uint32_t block_prefix(uint32_t v, uint32_t carry, uint32_t* wsum) {
  uint32_t pre = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(pre, o, 64);
    if ((threadIdx.x & 63) >= (unsigned)o) pre += t;
  }
  if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = pre;
  __syncthreads();
  uint32_t add = carry;
  for (int w = 0; w < (int)(threadIdx.x >> 6); w++) add += wsum[w];
  return pre + add;
}

// ---------------------------------------------------------------------------
// detect_edge (masks.c:54-100) from precomputed sums S[] along the scan axis.
//   bar k spans [b0 + k*step, b0 + k*step + size - 1] along the scan axis and
//   [c0, c1] across it; blackness_k = 255 - sum_k / count_pixels(clip(bar_k))
//   (count_pixels is |dx|+1 * |dy|+1 of the clipped, possibly inverted,
//   rectangle; the sum is 0 when that rectangle is empty).  The reference loop
//   runs k = 0,1,.. and continues while b_k >= (thr*total_k)/(k+1) && b_k != 0.
//   Guard: a bar entirely outside the image stops the scan when thr <= 1 (the
//   reference would loop forever there; DESIGN.md documents this).
// ---------------------------------------------------------------------------

__global__ void __launch_bounds__(256) k_edge_scan(const EdgeArgs* args, const uint32_t* sums,
                                                   int64_t sums_stride, int32_t* results) {
  const int s = blockIdx.y;
  const int job = blockIdx.x;
  const int64_t slot = (int64_t)s * gridDim.x + job;
  const EdgeArgs a = args[slot];
  if (!a.active) return;
  const uint32_t* S = sums + (int64_t)s * sums_stride + a.sums_offset;
  extern __shared__ uint32_t lds[];  // a.extent entries (launch: the largest extent)
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t carry;
  __shared__ int32_t stop_k;
  const int32_t n = a.extent;
  for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = S[i];
  if (threadIdx.x == 0) {
    carry = 0;
    stop_k = INT_MAX;
  }
  __syncthreads();
  // cross extent, clipped (the loop body runs iff cc0 <= cc1)
  const int32_t clo = imin(a.c0, a.c1), chi = imax(a.c0, a.c1);
  const int32_t cc0 = imax(clo, 0), cc1 = imin(chi, a.cross_extent - 1);
  const int32_t ccount = iabs(cc1 - cc0) + 1;
  const bool cross_out = chi < 0 || clo >= a.cross_extent;
  for (int32_t kb = 0; kb < (1 << 21); kb += blockDim.x) {
    const int32_t k = kb + (int32_t)threadIdx.x;
    const int32_t x0 = a.b0 + k * a.step, x1 = x0 + a.size - 1;
    const int32_t lo = imin(x0, x1), hi = imax(x0, x1);
    const int32_t cx0 = imax(lo, 0), cx1 = imin(hi, n - 1);
    uint64_t sum = 0;
    if (cx0 <= cx1 && cc0 <= cc1)
      for (int32_t x = cx0; x <= cx1; x++) sum += lds[x];
    const uint64_t cnt = (uint64_t)(uint32_t)((iabs(cx1 - cx0) + 1) * ccount);
    const uint32_t b = (uint8_t)(0xFFull - sum / cnt);  // blit.c:91-109
    const uint32_t total = block_prefix(b, carry, wsum);
    const uint32_t count = (uint32_t)k + 1;
    const bool cont = ((float)b >= ((a.threshold * total) / count)) && b != 0;
    const bool outside = hi < 0 || lo >= n || cross_out;
    const bool guard = outside && (a.threshold <= 1.0f || count >= (1u << 20));
    if (!cont || guard) atomicMin(&stop_k, k);
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) carry = total;
    __syncthreads();
    if (stop_k != INT_MAX) break;
  }
  if (threadIdx.x == 0) results[slot] = stop_k == INT_MAX ? (1 << 21) : stop_k + 1;
}

// The sums along the scan axis are staged in dynamic LDS sized to the largest
// extent (a static 64 KB array held a CU's LDS for the whole scan).
static size_t axis_lds(int32_t max_extent, const void* kernel) {
  const size_t b = sizeof(uint32_t) * (size_t)imax(max_extent, 1);
  allow_dynamic_lds(kernel, b);
  return b;
}

void launch_edge_scan(const EdgeArgs* args, int jobs_per_sheet, const uint32_t* sums,
                      int64_t sums_stride, int32_t* results, int count, hipStream_t st,
                      int32_t max_extent) {
  if (jobs_per_sheet <= 0 || count <= 0) return;
  hipLaunchKernelGGL(k_edge_scan, dim3(jobs_per_sheet, count), dim3(256),
                     axis_lds(max_extent, (const void*)k_edge_scan), st, args, sums, sums_stride,
                     results);
}

// ---------------------------------------------------------------------------
// detect_border_edge (masks.c:410-449): band k covers [lo + k*step, hi +
// k*step] (inclusive, as scanned; rows/cols outside the image count 0).
// result = k*|step| for the first k with count >= threshold while
// k*|step| < max_step, else 0.
// ---------------------------------------------------------------------------
// Counted rows may have a gap [gap0, gap1) (gap0 >= gap1: none): a band
// reaching into it before any band hits marks the sheet in need[] (the caller
// counts the gap and scans that sheet again); only (optional): the sheets to
// scan.
__global__ void __launch_bounds__(256) k_border_scan(const BorderEdgeArgs* args,
                                                     const uint32_t* sums, int64_t sums_stride,
                                                     int32_t* results, int32_t gap0, int32_t gap1,
                                                     int32_t* need, const int32_t* only) {
  const int s = blockIdx.y;
  const int job = blockIdx.x;
  if (only && !only[s]) return;
  const int64_t slot = (int64_t)s * gridDim.x + job;
  const BorderEdgeArgs a = args[slot];
  if (!a.active) return;
  const uint32_t* S = sums + (int64_t)s * sums_stride + a.sums_offset;
  extern __shared__ uint32_t lds[];  // a.extent entries (launch: the largest extent)
  __shared__ int32_t found;
  const int32_t n = a.extent;
  for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = S[i];
  if (threadIdx.x == 0) found = INT_MAX;
  __syncthreads();
  const int32_t ast = iabs(a.step);
  if (ast == 0) {
    // result never advances: the reference loops forever unless band 0 hits
    if (threadIdx.x == 0) {
      uint32_t c = 0;
      for (int32_t p = imax(a.lo, 0); p <= imin(a.hi, n - 1); p++) c += lds[p];
      results[slot] = 0;
      (void)c;
    }
    return;
  }
  const int32_t kmax = (a.max_step + ast - 1) / ast;  // k*|step| < max_step
  // found: 2 k for the first hit, 2 k + 1 when band k reaches the gap first
  for (int32_t kb = 0; kb < kmax; kb += blockDim.x) {
    const int32_t k = kb + (int32_t)threadIdx.x;
    if (k < kmax) {
      const int32_t lo = a.lo + k * a.step, hi = a.hi + k * a.step;
      const int32_t p0 = imax(lo, 0), p1 = imin(hi, n - 1);
      if (p0 <= p1 && p0 < gap1 && p1 >= gap0) {
        atomicMin(&found, 2 * k + 1);
      } else {
        uint32_t c = 0;
        for (int32_t p = p0; p <= p1; p++) c += lds[p];
        if (c >= (uint32_t)a.threshold) atomicMin(&found, 2 * k);
      }
    }
    __syncthreads();
    if (found != INT_MAX) break;
  }
  if (threadIdx.x == 0) {
    const bool gap = found != INT_MAX && (found & 1);
    if (gap) need[s] = 1;
    results[slot] = found == INT_MAX || gap ? 0 : (found >> 1) * ast;
  }
}

void launch_border_scan(const BorderEdgeArgs* args, int jobs_per_sheet, const uint32_t* sums,
                        int64_t sums_stride, int32_t* results, int count, hipStream_t st,
                        int32_t max_extent, int32_t gap0, int32_t gap1, int32_t* need,
                        const int32_t* only) {
  if (jobs_per_sheet <= 0 || count <= 0) return;
  if (gap0 < gap1 && !need) return;  // a gap needs somewhere to report
  hipLaunchKernelGGL(k_border_scan, dim3(jobs_per_sheet, count), dim3(256),
                     axis_lds(max_extent, (const void*)k_border_scan), st, args, sums, sums_stride,
                     results, gap0, gap1, need, only);
}

}  // namespace uph
