// kernels_deskew.hip — rotation detection (deskew.c:48-241).
//
// One workgroup per (sheet, edge, angle).  The reference walks a 1500-point
// virtual line inward one pixel per step, summing 255-max(rgb) under the line,
// until the accumulated blackness reaches 255*size*depth; the peak is the
// largest step-to-step increase.  Here the four waves split the line points
// and each lane owns one inward step of a 64-step chunk, so a wave reads 64
// consecutive pixels of one image row per point (one coalesced load) and the
// stopping rule is evaluated on the chunk with a wave prefix sum.
#include <climits>
#include <cmath>

#include "filters.h"

namespace uph {

__device__ __forceinline__ int iwave_prefix_excl(int v, int* total) {
  const int lane = threadIdx.x & 63;
  int pre = v;
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(pre, o, 64);
    if (lane >= o) pre += t;
  }
  *total = __shfl(pre, 63, 64);
  return pre - v;
}

// Geometry of one virtual scan line (detect_edge_rotation_peak,
// deskew.c:48-112): point count, depth limit and the float recurrence start.
struct LineSetup {
  int scan, maxDepth;
  float X, Y, stepX, stepY;
};

__device__ __forceinline__ LineSetup line_setup(const Rect& mask, const RotGeom& g, int sxh,
                                                int syv, float m) {
  LineSetup L;
  const int32_t mw = iabs(mask.x0 - mask.x1) + 1, mh = iabs(mask.y0 - mask.y1) + 1;
  int scan = g.scan_size, half, outer, mid, side;
  if (syv == 0) {
    if (scan == -1) scan = mh;
    scan = imin(imin(scan, 10000), mh);
    L.maxDepth = mw / 2;
    half = scan / 2;
    outer = (int)(fabsf(m) * half);
    mid = mh / 2;
    side = sxh > 0 ? mask.x0 - outer : mask.x1 + outer;
    L.X = side + half * m;
    L.Y = mask.y0 + mid - half;
    L.stepX = -m;
    L.stepY = 1.0;
  } else {
    if (scan == -1) scan = mw;
    scan = imin(imin(scan, 10000), mw);
    L.maxDepth = mh / 2;
    half = scan / 2;
    outer = (int)(fabsf(m) * half);
    mid = mw / 2;
    side = syv > 0 ? mask.x0 - outer : mask.x1 + outer;  // x-vertices (deskew.c:96-97)
    L.X = mask.x0 + mid - half;
    L.Y = side - (half * m);
    L.stepX = 1.0;
    L.stepY = -m;
  }
  L.scan = scan;
  return L;
}

// The point lists of every (sheet, edge, angle) line: one lane per line runs
// the float recurrence of deskew.c:107-112 in order.  Point i of line t is
// stored at pts[(2i + c) * nlines + t] (c = 0: x, 1: y) so a wave's stores
// are contiguous.
__global__ void __launch_bounds__(64) k_rot_points(RotGeom g, const RotTable* table,
                                                   const Rect* masks, const int32_t* mask_active,
                                                   int count, int32_t* pts) {
  const int na = table->nangles;
  const int nlines = count * g.nedges * na;
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= nlines) return;
  const int a = t % na, e = (t / na) % g.nedges, s = t / (na * g.nedges);
  if (mask_active && !mask_active[s]) return;
  const LineSetup L = line_setup(masks[s], g, g.edge_shift[e][0], g.edge_shift[e][1],
                                 table->slope[a]);
  float X = L.X, Y = L.Y;
  for (int i = 0; i < L.scan; i++) {
    pts[(int64_t)(2 * i) * nlines + t] = (int)X;
    pts[(int64_t)(2 * i + 1) * nlines + t] = (int)Y;
    X += L.stepX;
    Y += L.stepY;
  }
}

template <int FMT>
__global__ void __launch_bounds__(256) k_rot_peaks(PlaneRef img, RotGeom g, const RotTable* table,
                                                  const Rect* masks, const int32_t* mask_active,
                                                  int mask_index, int32_t* peaks,
                                                  const int32_t* lines, int count) {
  const int a = blockIdx.x, e = blockIdx.y, s = blockIdx.z;
  const int na = table->nangles;
  int32_t* out = peaks + (((int64_t)s * g.max_masks + mask_index) * 4 + e) * na + a;
  if (mask_active && !mask_active[s]) {
    if (threadIdx.x == 0) *out = 0;
    return;
  }
  const Rect mask = masks[s];
  const int sxh = g.edge_shift[e][0], syv = g.edge_shift[e][1];
  const float m = table->slope[a];
  const int maxAbs = (int)(255 * g.scan_size * g.scan_depth);
  const LineSetup LS = line_setup(mask, g, sxh, syv, m);
  const int scan = LS.scan, maxDepth = LS.maxDepth;
  extern __shared__ int32_t pts[];  // [scan] x, then [scan] y
  constexpr int kMaxWaves = 4;
  __shared__ int32_t part[kMaxWaves][64];
  __shared__ int32_t done_flag, result;
  if (scan <= 0) {
    if (threadIdx.x == 0) *out = 0;
    return;
  }
  int32_t* px = pts;
  int32_t* py = pts + scan;
  {
    const int nlines = count * g.nedges * na;
    const int t = (s * g.nedges + e) * na + a;
    for (int i = threadIdx.x; i < scan; i += blockDim.x) {
      px[i] = lines[(int64_t)(2 * i) * nlines + t];
      py[i] = lines[(int64_t)(2 * i + 1) * nlines + t];
    }
  }
  if (threadIdx.x == 0) {
    done_flag = 0;
    result = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint8_t* base = plane_ptr(img, s);
  const Rect nm = normalize(mask);
  int carry_acc = 0, last = 0, maxDiff = 0;  // wave 0 state
  if (syv == 0 && FMT == F_GRAY8) {
    // left/right edges of a gray plane: lane owns 4 consecutive depths of a
    // 256-depth chunk and reads them with two aligned dword loads per point
    // (a point's row is uniform across the wave, so rows outside the mask or
    // image are skipped with a scalar branch)
    const int32_t xlo = imax(nm.x0, 0), xhi = imin(nm.x1, g.W - 1);
    const int32_t ylo = imax(nm.y0, 0), yhi = imin(nm.y1, g.H - 1);
    const int iend = xlo <= xhi ? scan : 0;   // mask entirely off the image: all white
    const int64_t pitch = img.P.pitch;
    __shared__ int32_t part4[kMaxWaves][256];
    for (int d0 = 0; d0 < maxDepth; d0 += 256) {
      int acc[4] = {0, 0, 0, 0};
      const int32_t dl = d0 + 4 * lane;        // first depth of this lane
      // branch-free: a row outside the mask/image is read at a valid row and
      // masked, so the unrolled loads can all be in flight together
#pragma unroll 8
      for (int i = w; i < iend; i += nw) {
        const int32_t yr = __builtin_amdgcn_readfirstlane(py[i]);
        const bool rowok = yr >= ylo && yr <= yhi;
        const int32_t y = rowok ? yr : ylo;
        const int32_t xi = __builtin_amdgcn_readfirstlane(px[i]);
        // depth k of this lane is at column xi + sxh*(dl + k)
        const int32_t xs = sxh > 0 ? xi + dl : xi - dl - 3;   // lowest column of the 4
        // one unconditional aligned 8-byte window per lane (no divergent
        // branch around the loads, so the unrolled points' loads overlap);
        // every in-range column of the lane lies inside it
        const int32_t xa = imin(imax(xs, 0), (int32_t)pitch - 8) & ~3;
        const uint32_t* q = reinterpret_cast<const uint32_t*>(base + (int64_t)y * pitch + xa);
        const uint64_t V = ((uint64_t)q[1] << 32) | q[0];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int32_t x = sxh > 0 ? xs + k : xs + 3 - k;
          const bool ok = rowok && (uint32_t)(x - xlo) <= (uint32_t)(xhi - xlo);
          const int b = (int)((V >> ((8 * (x - xa)) & 63)) & 0xFF);
          acc[k] += (255 - b) & -(int)ok;  // arithmetic mask: the load is never sunk into a branch
        }
      }
#pragma unroll
      for (int k = 0; k < 4; k++) part4[w][4 * lane + k] = acc[k];
      __syncthreads();
      if (w == 0) {
        int B[4], pre[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          B[k] = 0;
          for (int q = 0; q < nw; q++) B[k] += part4[q][4 * lane + k];
          pre[k] = (k ? pre[k - 1] : 0) + B[k];
        }
        int tot;
        const int ex = carry_acc + iwave_prefix_excl(pre[3], &tot);
        // first depth (in order) that does not execute: before >= maxAbs or dep >= maxDepth
        int kfail = 4;
#pragma unroll
        for (int k = 3; k >= 0; k--) {
          const int before = ex + (k ? pre[k - 1] : 0);
          if (!(before < maxAbs && dl + k < maxDepth)) kfail = k;
        }
        const unsigned long long F = __ballot(kfail < 4);
        const int fl = F ? __ffsll((long long)F) - 1 : 64;
        const int stop = fl < 64 ? 4 * fl + __shfl(kfail, fl, 64) : 256;
        const int up = __shfl_up(B[3], 1, 64);
        int prev = lane == 0 ? last : up;
        int md = INT_MIN;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (4 * lane + k < stop) md = max(md, B[k] - prev);
          prev = B[k];
        }
        for (int o = 32; o > 0; o >>= 1) md = max(md, __shfl_xor(md, o, 64));
        if (md > maxDiff) maxDiff = md;  // `if (diff >= maxDiff) maxDiff = diff`
        if (stop < 256) {
          if (lane == 0) {
            result = (d0 + stop) < maxDepth ? maxDiff : 0;
            done_flag = 1;
          }
        } else {
          carry_acc += tot;
          last = __shfl(B[3], 63, 64);
        }
      }
      __syncthreads();
      if (done_flag) break;
    }
    if (threadIdx.x == 0) *out = done_flag ? result : 0;
    return;
  }
  for (int d0 = 0; d0 < maxDepth; d0 += 64) {
    const int dep = d0 + lane;
    int acc = 0;
    // branch-free gather (out-of-mask/out-of-image points read pixel (0,0)
    // and contribute 0, i.e. get_pixel's white), unrolled so several loads
    // per lane are in flight
#pragma unroll 8
    for (int i = w; i < scan; i += nw) {
      const int32_t x = px[i] + sxh * dep, y = py[i] + syv * dep;
      const bool ok = (x >= nm.x0) & (x <= nm.x1) & (y >= nm.y0) & (y <= nm.y1) & (x >= 0) &
                      (y >= 0) & (x < g.W) & (y < g.H);
      const Px p = load_px_row<FMT>(base + (int64_t)(ok ? y : 0) * img.P.pitch, ok ? x : 0);
      acc += (255 - (int)dark_of(p)) & -(int)ok;
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0) {
      int B = 0;
      for (int q = 0; q < nw; q++) B += part[q][lane];
      int tot;
      const int before = carry_acc + iwave_prefix_excl(B, &tot);
      const bool exec = before < maxAbs && dep < maxDepth;
      const unsigned long long X_ = __ballot(!exec);
      const int stop = X_ ? __ffsll((long long)X_) - 1 : 64;
      // the permute runs on the whole wave: a lane reading an inactive lane's
      // register gets no defined value
      const int up = __shfl_up(B, 1, 64);
      const int prevB = lane == 0 ? last : up;
      const int diff = B - prevB;
      int md = lane < stop ? diff : INT_MIN;
      for (int o = 32; o > 0; o >>= 1) md = max(md, __shfl_xor(md, o, 64));
      if (md > maxDiff) maxDiff = md;  // `if (diff >= maxDiff) maxDiff = diff`
      if (stop < 64) {
        if (lane == 0) {
          result = (d0 + stop) < maxDepth ? maxDiff : 0;
          done_flag = 1;
        }
      } else {
        carry_acc += tot;
        last = __shfl(B, 63, 64);
      }
    }
    __syncthreads();
    if (done_flag) break;
  }
  if (threadIdx.x == 0) *out = done_flag ? result : 0;
}

size_t rotation_lines_bytes(int count, int nedges, int nangles, int max_scan) {
  return sizeof(int32_t) * 2 * (size_t)(max_scan > 0 ? max_scan : 1) * count * nedges * nangles;
}

void launch_rotation_peaks(const PlaneRef& img, const RotGeom& g, const RotTable* table,
                           const Rect* masks, const int32_t* mask_active, int mask_index,
                           int32_t* peaks, int count, hipStream_t st, int nangles,
                           int max_scan, int32_t* lines) {
  if (g.nedges <= 0 || nangles <= 0) return;
  const int nlines = count * g.nedges * nangles;
  hipLaunchKernelGGL(k_rot_points, dim3((nlines + 63) / 64), dim3(64), 0, st, g, table, masks,
                     mask_active, count, lines);
  dim3 grid(nangles, g.nedges, count);
  const size_t lds = sizeof(int32_t) * 2 * (size_t)(max_scan > 0 ? max_scan : 1);
  if (lds > 64 * 1024) {
    hipFuncSetAttribute((const void*)k_rot_peaks<F_GRAY8>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)k_rot_peaks<F_Y400A>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipFuncSetAttribute((const void*)k_rot_peaks<F_RGB24>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  }
  switch (img.P.fmt) {
    case F_GRAY8:
      hipLaunchKernelGGL(k_rot_peaks<F_GRAY8>, grid, dim3(256), lds, st, img, g, table, masks,
                         mask_active, mask_index, peaks, lines, count);
      break;
    case F_Y400A:
      hipLaunchKernelGGL(k_rot_peaks<F_Y400A>, grid, dim3(256), lds, st, img, g, table, masks,
                         mask_active, mask_index, peaks, lines, count);
      break;
    default:
      hipLaunchKernelGGL(k_rot_peaks<F_RGB24>, grid, dim3(256), lds, st, img, g, table, masks,
                         mask_active, mask_index, peaks, lines, count);
      break;
  }
}

}  // namespace uph

namespace uph {

int rotation_angles(const UphipDeskewParameters& p, RotTable* t) {
  // for (rotation = 0.0; rotation <= range; rotation = (rotation >= 0.0) ?
  //      -(rotation + step) : -rotation)   (deskew.c:158-160), m = tanf (:161)
  int n = 0;
  for (float r = 0.0; r <= p.deskewScanRangeRad;
       r = (r >= 0.0) ? -(r + p.deskewScanStepRad) : -r) {
    if (n >= kMaxAngles) return -1;
    t->angle[n] = r;
    t->slope[n] = tanf(r);
    n++;
  }
  t->nangles = n;
  return n;
}

float combine_edge_rotations(const float* rotation, int count, float deviation_rad) {
  // detect_rotation_cpu, deskew.c:219-240
  float total = 0.0;
  for (int i = 0; i < count; i++) total += rotation[i];
  float average = total / count;
  total = 0.0;
  // glibc powf through a pointer, as the reference's default -O0 build calls
  // it (an optimising compiler would fold powf(x, 2) into x*x)
  static float (*volatile pw)(float, float) = powf;
  for (int i = 0; i < count; i++) total += pw(rotation[i] - average, 2);
  float deviation = sqrtf(total);
  return deviation <= deviation_rad ? average : 0.0f;
}

}  // namespace uph
