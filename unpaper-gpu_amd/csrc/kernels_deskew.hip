// kernels_deskew.hip — rotation detection (deskew.c:48-241).
//
// The reference walks, for every angle and enabled edge, a virtual line of up
// to 1500 points inward one pixel per step, summing 255-max(rgb) under the
// line, until the accumulated blackness reaches 255*size*depth; the peak is
// the largest step-to-step increase (detect_edge_rotation_peak).
//
// For the left/right edges (the default) the line's rows do not depend on
// the angle: point i sits on row Ystart+i for every angle, only its column
// (int)X_i differs.  So all angles and the first kDepth steps read one band
// of columns beside the mask edge.  The fast path is
//   k_rot_points  the float recurrence X += -m of every line (deskew.c:
//                 107-112) in closed form per binade -> a few segments per
//                 line (point i of a segment: X = T + (i - i0) d, exact);
//   k_rot_band_g  one workgroup per 128-row slice of a (sheet, edge): the
//                 slice's band is staged in LDS as per-column prefix sums of
//                 the blackness, then every angle x kDepth steps is summed
//                 run by run (two prefix entries per run) -> partials;
//   k_rot_final   one wave per line: slice partials -> blackness per step,
//                 then the reference's stopping rule and peak, exactly.
// Lines that do not stop within kDepth steps, top/bottom edges (rows move
// with the step) and bands too wide for LDS (very large angle ranges) are
// flagged and walked by k_rot_line, a direct per-line restatement.
#include <climits>
#include <mutex>
#include <vector>
#include <cmath>

#include "filters.h"
#include "libm_glibc.h"

namespace uph {

constexpr int kDepth = 128;        // steps covered by the band path (2 per lane)
constexpr int kSliceRows = 128;    // rows per band slice
constexpr int kBandCapMax = 384;   // band columns at most (LDS: 256 bytes per column)

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

// Scratch layout of one launch:
//   segs   [nlines][kLineSegs]  int4 {i0, n, T, d}: points i0 .. i0+n of a
//                               left/right line have column (int)(T + (i-i0) d)
//                               (T, d floats, the sum exact: it is the
//                               recurrence's float X_i)
//   nseg   [nlines]             segments of the line (0: none, walked directly)
//   ends   [nlines][2]          first and last column of the line
//   part   [nlines][nslices][kDepth]  band slice sums, u16 (<= 128 * 255)
//   flag   [nlines]             1 = walk the line directly (k_rot_line)
//   state  [nlines][4]          band result after kDepth steps: accumulated,
//                               last step's blackness, peak, valid
//   list   [nlines]             the flagged lines (k_rot_line's work list)
//   nlist  [1]                  their count (zeroed before k_rot_points)
constexpr int kLineSegs = 32;  // a line with more (it passes near X = 0) is walked directly
struct RotScratch {
  int4* segs;
  int32_t *nseg, *ends;
  uint16_t* part;
  int32_t *flag, *state, *list, *nlist;
  int32_t *blo, *bhi;  // per (sheet, edge): the least / greatest column of its lines' ends
};

__host__ __device__ static inline int rot_slices(int max_scan) { return (max_scan + kSliceRows - 1) / kSliceRows; }

// int32 words of each array (part: u16 pairs; kDepth is even)
__host__ __device__ static inline RotScratch rot_scratch(int32_t* base, int nlines, int max_scan) {
  RotScratch r;
  const int64_t ms = max_scan > 0 ? max_scan : 1;
  const int64_t ns = (ms + kSliceRows - 1) / kSliceRows;
  r.segs = reinterpret_cast<int4*>(base);
  r.nseg = base + (int64_t)nlines * kLineSegs * 4;
  r.ends = r.nseg + nlines;
  r.part = reinterpret_cast<uint16_t*>(r.ends + 2 * (int64_t)nlines);
  r.flag = r.ends + 2 * (int64_t)nlines + (int64_t)nlines * ns * (kDepth / 2);
  r.state = r.flag + nlines;
  r.list = r.state + 4 * (int64_t)nlines;
  r.nlist = r.list + nlines;
  r.blo = r.nlist + 1;           // indexed by sheet * nedges + edge (< nlines)
  r.bhi = r.blo + nlines;
  return r;
}

// column of point i of a left/right line from its segments (sorted by i0,
// covering 0 .. scan-1): exact, see k_rot_points
__device__ __forceinline__ int32_t seg_col(const int4* sg, int nsg, int i) {
  float T = 0.0f, d = 0.0f;
  int b = 0;
  for (int q = 0; q < nsg; q++) {
    const int4 v = sg[q];
    if (v.x > i) break;
    T = __int_as_float(v.z);
    d = __int_as_float(v.w);
    b = v.x;
  }
  return (int)fmaf((float)(i - b), d, T);
}

const int32_t* rotation_line_flags(const int32_t* lines, int nlines, int max_scan) {
  return rot_scratch(const_cast<int32_t*>(lines), nlines, max_scan).flag;
}

size_t rotation_lines_bytes(int count, int nedges, int nangles, int max_scan) {
  const int64_t nlines = (int64_t)count * nedges * nangles;
  const int64_t ms = max_scan > 0 ? max_scan : 1;
  const int64_t ns = (ms + kSliceRows - 1) / kSliceRows;
  return sizeof(int32_t) * (size_t)(nlines * kLineSegs * 4 + nlines + 2 * nlines +
                                    nlines * ns * (kDepth / 2) + nlines + 4 * nlines + nlines + 1 +
                                    2 * nlines);
}

// ---- k_rot_points: the points of every left/right line --------------------
// The reference builds a line by the float recurrence X_{i+1} = fl(X_i + s)
// (deskew.c:107-112).  While X stays inside one binade [2^(E-1), 2^E) the
// rounding of X_i + s to the binade's ulp u is X_i + round_u(s): the same
// increment d every step (for a tie, s/u a half-integer, the even multiple
// wins, constant from an even X_i/u on), so X_i = T + k*d exactly for a whole
// run of steps, whose length follows from integer arithmetic in units of u.
// A thread per line splits it into such segments, with one explicit float
// step at each binade change, odd-tie start or X = 0, and stores them (the
// band and the direct walk evaluate a point's column from them: T, d and
// every T + k d are floats, so fmaf(k, d, T) is exact).  A line with more
// than kLineSegs segments (one passing near X = 0) is walked directly.
__global__ void __launch_bounds__(256) k_rot_points(RotGeom g, const RotTable* table,
                                                    const Rect* masks, const int32_t* mask_active,
                                                    int count, RotScratch R) {
  const int na = table->nangles;
  const int nlines = count * g.nedges * na;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  // the block's (sheet, edge) column ranges, reduced in LDS first (the lines
  // of one pair are consecutive: <= 256 pairs a block)
  __shared__ int32_t slo[256], shi[256];
  const int se_base = (int)(blockIdx.x * blockDim.x) / na;
  slo[threadIdx.x] = INT_MAX;
  shi[threadIdx.x] = INT_MIN;
  __syncthreads();
  [&] {  // one line (returns leave the lambda; every thread reaches the barrier below)
  if (t >= nlines) return;
  const int a = t % na, e = (t / na) % g.nedges, s = t / (na * g.nedges);
  const bool act = !(mask_active && !mask_active[s]);
  R.state[4 * t + 3] = 0;
  if (!act || g.edge_shift[e][1] != 0) {
    R.ends[2 * t] = 0;
    R.ends[2 * t + 1] = 0;
    R.nseg[t] = 0;
    R.flag[t] = 1;
    if (act) R.list[atomicAdd(R.nlist, 1)] = t;  // a top/bottom edge: walked directly
    return;
  }
  const LineSetup L = line_setup(masks[s], g, g.edge_shift[e][0], 0, table->slope[a]);
  const int scan = L.scan;
  int4* sg = R.segs + (int64_t)t * kLineSegs;
  int ns = 0, last = 0;
  bool over = false;
  float X = L.X;
  const float st = L.stepX;
  int i = 0;
  while (scan > 0) {
    if (ns >= kLineSegs) {
      over = true;
      break;
    }
    const float sign = X > 0.0f ? 1.0f : -1.0f;
    const double T = (double)fabsf(X), sig = (double)st * (double)sign;
    int64_t nn = 0;
    double du = 0.0;
    if (X != 0.0f) {
      int E;
      frexpf(fabsf(X), &E);  // |X| = m * 2^E, m in [0.5, 1)
      if (E < -100) {        // u would leave the float range: walk directly
        over = true;
        break;
      }
      const double lo = ldexp(1.0, E - 1), hi = ldexp(1.0, E), u = ldexp(1.0, E - 24);
      // divisions by u are exact scalings (u is a power of two)
      const double q = ldexp(sig, 24 - E);
      const double fqd = floor(q);
      const int64_t fq = (int64_t)fqd;
      // A tie (q = fq + 1/2) rounds to the even multiple of u: from an even
      // |X|/u the increment is then always the even one of fq, fq + 1; from
      // an odd one, one explicit step first.
      const bool tie = q - fqd == 0.5;
      if (!tie || !(((int64_t)ldexp(T, 24 - E)) & 1)) {
        const int64_t dq = tie ? (fq & 1 ? fq + 1 : fq) : (int64_t)floor(q + 0.5);
        // units of u left to the binade's ends: < 2^24
        const int64_t H = (int64_t)ldexp(hi - T, 24 - E), G = (int64_t)ldexp(T - lo, 24 - E);
        const int64_t rem = scan - 1 - i;  // steps still to take
        // c / d for 0 <= c < 2^24, d >= 1 in 32 bits (c / d = 0 when d > c)
        auto div24 = [](int64_t c, int64_t d) -> int64_t {
          return d > c ? 0 : (int64_t)((uint32_t)c / (uint32_t)d);
        };
        // steps k = 1.. whose exact sum X_{k-1} + s stays in [lo, hi)
        if (dq > 0) {
          const int64_t c = H - fq - 1;
          nn = c >= 0 ? div24(c, dq) + 1 : 0;
        } else if (dq < 0) {
          const int64_t c = G + fq;
          nn = c >= 0 ? div24(c, -dq) + 1 : 0;
        } else {
          nn = (q >= 0.0 || G >= 1) ? rem : 0;
        }
        if (nn > rem) nn = rem;
        du = (double)dq * u;  // s rounded to u: a float (s itself, or < 2^24 units of u)
      }
    }
    const float Ts = sign * (float)T, ds = sign * (float)du;
    sg[ns++] = make_int4(i, (int32_t)nn, __float_as_int(Ts), __float_as_int(ds));
    i += (int)nn;
    if (i >= scan - 1) {
      last = (int)fmaf((float)nn, ds, Ts);
      break;
    }
    // one explicit step (binade change, tie or zero)
    X = sign * (float)(T + (double)nn * du) + st;
    i++;
  }
  const int first = scan > 0 ? (int)L.X : 0;  // point 0 is the start value itself
  R.ends[2 * t] = first;
  R.ends[2 * t + 1] = over ? first : last;
  // the (sheet, edge)'s column range over all its lines (band_range)
  const int se = t / na, lo = over ? first : imin(first, last), hi = over ? first : imax(first, last);
  atomicMin(&slo[se - se_base], lo);
  atomicMax(&shi[se - se_base], hi);
  R.nseg[t] = over ? 0 : ns;
  R.flag[t] = over;
  if (over) R.list[atomicAdd(R.nlist, 1)] = t;
  }();
  __syncthreads();
  const int tl = imin(nlines, (int)((blockIdx.x + 1) * blockDim.x)) - 1;
  const int ng = tl >= 0 ? tl / na - se_base + 1 : 0;
  if ((int)threadIdx.x < ng && slo[threadIdx.x] <= shi[threadIdx.x]) {
    atomicMin(&R.blo[se_base + threadIdx.x], slo[threadIdx.x]);
    atomicMax(&R.bhi[se_base + threadIdx.x], shi[threadIdx.x]);
  }
}

// Band of one (sheet, edge): columns [bx0, bx0 + bw) cover every point of
// every angle for steps 0..kDepth-1.  Returns false when it does not fit.
__device__ __forceinline__ bool band_range(const RotScratch& R, int tbase, int na, int sxh,
                                           int band_cap, int32_t* bx0, int32_t* bw) {
  const int se = tbase / na;
  int32_t lo = R.blo[se], hi = R.bhi[se];
  if (sxh > 0) hi += kDepth - 1;
  else lo -= kDepth - 1;
  *bx0 = lo;
  *bw = hi - lo + 1;
  return *bw <= band_cap && lo <= hi;
}

// ---- k_rot_band: slice sums of every angle x kDepth steps -----------------
// Along a slice a line's column changes only where (int)X steps, so it is a
// few vertical runs (1 + 128*|m| at most).  The slice's band is staged as
// per-column prefix sums over its rows (16-bit: 128 * 255 fits), and every
// (angle, depth) sum is a difference of two prefix entries per run.
constexpr int kBandThreads = 512;
__global__ void __launch_bounds__(kBandThreads, 4)
    k_rot_band_g(PlaneRef img, RotGeom g, const RotTable* table, const Rect* masks,
                 const int32_t* mask_active, int count, int max_scan, RotScratch R, int fmt,
                 int band_cap) {
  const int sl = blockIdx.x, e = blockIdx.y, s = blockIdx.z;
  const int na = table->nangles;
  const int sxh = g.edge_shift[e][0];
  if (g.edge_shift[e][1] != 0 || (mask_active && !mask_active[s])) return;
  const Rect mask = masks[s];
  const LineSetup LS = line_setup(mask, g, sxh, 0, 0.0f);  // scan, Ystart: angle independent
  const int i0 = sl * kSliceRows, i1 = imin(LS.scan, i0 + kSliceRows);
  if (i0 >= i1) return;
  const int tbase = (s * g.nedges + e) * na;
  int32_t bx0, bw;
  if (!band_range(R, tbase, na, sxh, band_cap, &bx0, &bw)) return;  // k_rot_final flags the lines
  // pre[r * bw + c]: blackness of rows 0..r of column c; the raw bytes are
  // staged first in the upper half
  // dynamic LDS: kSliceRows * band_cap entries (the launch sizes band_cap
  // from the angle range, so two slices fit a CU at the default range)
  extern __shared__ __attribute__((aligned(16))) uint16_t pre[];
  uint8_t* raw = reinterpret_cast<uint8_t*>(pre) + kSliceRows * bw;
  const Rect nm = normalize(mask);
  const int32_t xlo = imax(nm.x0, 0), xhi = imin(nm.x1, g.W - 1);
  const int32_t ylo = imax(nm.y0, 0), yhi = imin(nm.y1, g.H - 1);
  const int32_t ystart = (int32_t)LS.Y;  // exact: integer start, +1.0 per point
  const uint8_t* base = plane_ptr(img, s);
  const int rows = i1 - i0;
  // blackness 255-max(rgb) of in-mask, in-image pixels (0 elsewhere,
  // get_pixel's white); a wave per row, lanes along it (no index division),
  // unconditional clamped loads masked arithmetically, all of a row's in
  // flight
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int kPer = kBandCapMax / 64;
    for (int r = w; r < rows; r += kBandThreads / 64) {
      const int32_t y = ystart + i0 + r;
      const bool rok = (y >= ylo) & (y <= yhi);
      const uint8_t* row = base + (int64_t)(rok ? y : ylo) * img.P.pitch;
      uint8_t v[kPer];
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        const int c = lane + 64 * k;
        const int32_t x = bx0 + c;
        const bool ok = rok & (c < bw) & (x >= xlo) & (x <= xhi);
        const int32_t xo = ok ? x : xlo;
        uint32_t d;
        if (fmt == F_GRAY8) d = row[xo];
        else if (fmt == F_Y400A) d = row[2 * xo];
        else d = dark_of(load_px_row<F_RGB24>(row, xo));
        v[k] = (uint8_t)((255 - d) & -(int)ok);
      }
#pragma unroll
      for (int k = 0; k < kPer; k++) {
        const int c = lane + 64 * k;
        if (c < bw) raw[r * bw + c] = v[k];
      }
    }
  }
  __syncthreads();
  // column prefix sums: one thread per column, 32 rows at a time.  Prefix
  // row r (bytes [2 r bw, 2 r bw + 2 bw)) overwrites raw rows 2r-128 and
  // 2r-127 only, which every thread has read by then: each chunk is read
  // out before the barrier and written after it.
  const int c = threadIdx.x;
  uint32_t acc = 0;
  for (int k0 = 0; k0 < kSliceRows; k0 += 32) {
    uint32_t colv[8];
    if (c < bw) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        uint32_t wv = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int r = k0 + 4 * k + j;
          wv |= (r < rows ? (uint32_t)raw[r * bw + c] : 0u) << (8 * j);
        }
        colv[k] = wv;
      }
    }
    __syncthreads();
    if (c < bw) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int r = k0 + 4 * k + j;
          acc += (colv[k] >> (8 * j)) & 0xFFu;
          if (r < rows) pre[r * bw + c] = (uint16_t)acc;
        }
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int nw = kBandThreads / 64;
  const int32_t o0 = sxh * lane - bx0, o1 = sxh * (lane + 64) - bx0;
  const int ns = rot_slices(max_scan);
  for (int a = w; a < na; a += nw) {
    const int t = __builtin_amdgcn_readfirstlane(tbase + a);
    // the slice's columns, two rows per lane (from the line's segments that
    // overlap the slice); run starts by ballot
    int32_t cA = 0, cB = 0;
    {
      // lane q holds segment q (all loads in flight at once); each lane then
      // picks the last segment starting at or before its rows
      const int nsg = __builtin_amdgcn_readfirstlane(R.nseg[t]);
      const int4 mine = lane < nsg ? R.segs[(int64_t)t * kLineSegs + lane] : make_int4(INT_MAX, 0, 0, 0);
      const int iA = i0 + lane, iB = i0 + 64 + lane;
      // the segment holding row i0 (uniform), and whether it holds the slice
      int q0 = 0;
      while (q0 + 1 < nsg && __builtin_amdgcn_readlane(mine.x, q0 + 1) <= i0) q0++;
      const int nxt = q0 + 1 < nsg ? __builtin_amdgcn_readlane(mine.x, q0 + 1) : INT_MAX;
      if (nxt >= i1) {  // one segment: its values are wave-uniform
        const int b = __builtin_amdgcn_readlane(mine.x, q0);
        const float T = __int_as_float(__builtin_amdgcn_readlane(mine.z, q0));
        const float d = __int_as_float(__builtin_amdgcn_readlane(mine.w, q0));
        if (lane < rows) cA = (int)fmaf((float)(iA - b), d, T);
        if (lane + 64 < rows) cB = (int)fmaf((float)(iB - b), d, T);
      } else {
        int qA = q0, qB = q0;
        for (int q = q0 + 1; q < nsg; q++) {
          const int s0 = __builtin_amdgcn_readlane(mine.x, q);
          if (s0 >= i1) break;  // uniform: starts after the slice
          qA = iA >= s0 ? q : qA;
          qB = iB >= s0 ? q : qB;
        }
        const int bA = __shfl(mine.x, qA, 64), bB = __shfl(mine.x, qB, 64);
        const float TA = __int_as_float(__shfl(mine.z, qA, 64)), dA = __int_as_float(__shfl(mine.w, qA, 64));
        const float TB = __int_as_float(__shfl(mine.z, qB, 64)), dB = __int_as_float(__shfl(mine.w, qB, 64));
        if (lane < rows) cA = (int)fmaf((float)(iA - bA), dA, TA);
        if (lane + 64 < rows) cB = (int)fmaf((float)(iB - bB), dB, TB);
      }
    }
    const int32_t upA = __shfl_up(cA, 1, 64), upB = __shfl_up(cB, 1, 64);
    const int32_t lastA = __builtin_amdgcn_readlane(cA, 63);
    const bool stA = lane < rows && (lane == 0 || upA != cA);
    const bool stB = lane + 64 < rows && (lane == 0 ? lastA != cB : upB != cB);
    unsigned long long MA = __ballot(stA), MB = __ballot(stB);
    int acc0 = 0, acc1 = 0;
    int rs = 0;
    int32_t x = __builtin_amdgcn_readlane(cA, 0);
    MA &= MA - 1;  // row 0 starts the first run
    for (;;) {
      int re;  // end (exclusive) of the run starting at rs
      int32_t nx = 0;
      if (MA) {
        re = __ffsll((long long)MA) - 1;
        nx = __builtin_amdgcn_readlane(cA, re);
        MA &= MA - 1;
      } else if (MB) {
        const int b = __ffsll((long long)MB) - 1;
        re = 64 + b;
        nx = __builtin_amdgcn_readlane(cB, b);
        MB &= MB - 1;
      } else {
        re = rows;
      }
      const uint16_t* pe = pre + (re - 1) * bw + x;
      acc0 += pe[o0];
      acc1 += pe[o1];
      if (rs > 0) {
        const uint16_t* ps = pre + (rs - 1) * bw + x;
        acc0 -= ps[o0];
        acc1 -= ps[o1];
      }
      if (re >= rows) break;
      rs = re;
      x = nx;
    }
    uint16_t* P = R.part + ((int64_t)t * ns + sl) * kDepth;
    P[lane] = (uint16_t)acc0;
    P[lane + 64] = (uint16_t)acc1;
  }
}

// ---- k_rot_final: the stopping rule on the summed steps, one wave per line --
__global__ void __launch_bounds__(256) k_rot_final(RotGeom g, const RotTable* table,
                                                   const Rect* masks, const int32_t* mask_active,
                                                   int mask_index, int32_t* peaks, int count,
                                                   int max_scan, RotScratch R, int band_cap) {
  const int na = table->nangles;
  const int nlines = count * g.nedges * na;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= nlines) return;
  const int a = t % na, e = (t / na) % g.nedges, s = t / (na * g.nedges);
  int32_t* out = peaks + (((int64_t)s * g.max_masks + mask_index) * 4 + e) * na + a;
  if (mask_active && !mask_active[s]) {
    if (lane == 0) *out = 0;
    return;
  }
  if (R.flag[t]) return;  // top/bottom edge: k_rot_line
  const int sxh = g.edge_shift[e][0];
  const LineSetup LS = line_setup(masks[s], g, sxh, 0, table->slope[a]);
  int32_t bx0, bw;
  if (LS.scan <= 0) {
    if (lane == 0) *out = 0;
    return;
  }
  if (!band_range(R, (s * g.nedges + e) * na, na, sxh, band_cap, &bx0, &bw)) {
    if (lane == 0) {
      R.flag[t] = 1;
      R.list[atomicAdd(R.nlist, 1)] = t;
    }
    return;
  }
  const int ns = rot_slices(max_scan), nsl = (LS.scan + kSliceRows - 1) / kSliceRows;
  int B[2] = {0, 0};
#pragma unroll 4
  for (int q = 0; q < nsl; q++) {
    // steps 2 lane (low half) and 2 lane + 1 (high half) of slice q
    const uint32_t v = reinterpret_cast<const uint32_t*>(R.part + ((int64_t)t * ns + q) * kDepth)[lane];
    B[0] += (int)(v & 0xFFFFu);
    B[1] += (int)(v >> 16);
  }
  // steps 2*lane, 2*lane+1 (deskew.c:114-146)
  const int maxAbs = (int)(255 * g.scan_size * g.scan_depth);
  const int pre1 = B[0] + B[1];
  int tot;
  const int ex = iwave_prefix_excl(pre1, &tot);
  int kfail = 2;
  for (int k = 1; k >= 0; k--) {
    const int before = ex + (k ? B[0] : 0);
    if (!(before < maxAbs && 2 * lane + k < LS.maxDepth)) kfail = k;
  }
  const unsigned long long F = __ballot(kfail < 2);
  if (!F) {
    // still accumulating after kDepth steps: k_rot_line continues the walk
    // from step kDepth with the loop state reached here
    const int up1 = __shfl_up(B[1], 1, 64);
    const int prev0 = lane == 0 ? 0 : up1;
    int md = max(B[0] - prev0, B[1] - B[0]);
    for (int o = 32; o > 0; o >>= 1) md = max(md, __shfl_xor(md, o, 64));
    const int last = __shfl(B[1], 63, 64);
    if (lane == 0) {
      R.state[4 * t] = tot;
      R.state[4 * t + 1] = last;
      R.state[4 * t + 2] = md > 0 ? md : 0;
      R.state[4 * t + 3] = 1;
      R.flag[t] = 1;
      R.list[atomicAdd(R.nlist, 1)] = t;
    }
    return;
  }
  const int fl = __ffsll((long long)F) - 1;
  const int stop = 2 * fl + __shfl(kfail, fl, 64);
  const int up = __shfl_up(B[1], 1, 64);
  int prev = lane == 0 ? 0 : up;  // `last` starts at 0
  int md = INT_MIN;
  for (int k = 0; k < 2; k++) {
    if (2 * lane + k < stop) md = max(md, B[k] - prev);
    prev = B[k];
  }
  for (int o = 32; o > 0; o >>= 1) md = max(md, __shfl_xor(md, o, 64));
  const int maxDiff = md > 0 ? md : 0;  // maxDiff starts at 0, `diff >= maxDiff`
  if (lane == 0) *out = stop < LS.maxDepth ? maxDiff : 0;
}

// ---- k_rot_line: direct walk of one flagged line (any edge) ---------------
template <int FMT>
__device__ void walk_line(PlaneRef img, const RotGeom& g, const RotTable* table, const Rect* masks,
                          int mask_index, int32_t* peaks, int a, int e, int s, int t,
                          int max_scan, const RotScratch& R);

constexpr int kWalkThreads = 1024;  // 16 waves share a walked line's points
template <int FMT>
__global__ void __launch_bounds__(kWalkThreads) k_rot_line(PlaneRef img, RotGeom g, const RotTable* table,
                                                  const Rect* masks, const int32_t* mask_active,
                                                  int mask_index, int32_t* peaks, int count,
                                                  int max_scan, RotScratch R) {
  const int na = table->nangles;
  (void)count;
  // grid-strided over the work list of flagged lines (k_rot_points,
  // k_rot_final append them): an empty list costs one load per block
  const int n = __builtin_amdgcn_readfirstlane(*R.nlist);
  for (int q = blockIdx.x; q < n; q += gridDim.x) {
    const int t = __builtin_amdgcn_readfirstlane(R.list[q]);
    const int a = t % na, e = (t / na) % g.nedges, s = t / (na * g.nedges);
    if (mask_active && !mask_active[s]) continue;
    walk_line<FMT>(img, g, table, masks, mask_index, peaks, a, e, s, t, max_scan, R);
    __syncthreads();  // the block's LDS is reused by its next line
  }
}

template <int FMT>
__device__ void walk_line(PlaneRef img, const RotGeom& g, const RotTable* table, const Rect* masks,
                          int mask_index, int32_t* peaks, int a, int e, int s, int t,
                          int max_scan, const RotScratch& R) {
  const int na = table->nangles;
  int32_t* out = peaks + (((int64_t)s * g.max_masks + mask_index) * 4 + e) * na + a;
  const Rect mask = masks[s];
  const int sxh = g.edge_shift[e][0], syv = g.edge_shift[e][1];
  const LineSetup LS = line_setup(mask, g, sxh, syv, table->slope[a]);
  const int scan = LS.scan, maxDepth = LS.maxDepth;
  const int maxAbs = (int)(255 * g.scan_size * g.scan_depth);
  extern __shared__ int32_t pts[];  // [scan] x, then [scan] y
  constexpr int kWaves = kWalkThreads / 64;
  __shared__ int32_t part[kWaves][64];
  __shared__ int32_t done_flag, result;
  if (scan <= 0) {
    if (threadIdx.x == 0) *out = 0;
    return;
  }
  int32_t* px = pts;
  int32_t* py = pts + scan;
  // a left/right line continues from the band's state after kDepth steps,
  // with the point lists k_rot_points built; others start from scratch
  const bool resume = R.state[4 * t + 3] != 0;
  const int nsg = syv == 0 ? R.nseg[t] : 0;
  __shared__ int4 segs_s[kLineSegs];
  if (nsg > 0) {
    if ((int)threadIdx.x < nsg) segs_s[threadIdx.x] = R.segs[(int64_t)t * kLineSegs + threadIdx.x];
    __syncthreads();
    const int32_t ystart = (int32_t)LS.Y;  // rows: Ystart + i exactly
    for (int i = threadIdx.x; i < scan; i += blockDim.x) {
      px[i] = seg_col(segs_s, nsg, i);
      py[i] = ystart + i;
    }
  } else if (threadIdx.x == 0) {
    // the float recurrence of deskew.c:107-112, in order
    float X = LS.X, Y = LS.Y;
    for (int i = 0; i < scan; i++) {
      px[i] = (int)X;
      py[i] = (int)Y;
      X += LS.stepX;
      Y += LS.stepY;
    }
  }
  if (threadIdx.x == 0) {
    done_flag = 0;
    result = 0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint8_t* base = plane_ptr(img, s);
  const Rect nm = normalize(mask);
  int carry_acc = 0, last = 0, maxDiff = 0;  // wave 0 state
  int dstart = 0;
  if (resume) {
    carry_acc = R.state[4 * t];
    last = R.state[4 * t + 1];
    maxDiff = R.state[4 * t + 2];
    dstart = kDepth;
  }
  for (int d0 = dstart; d0 < maxDepth; d0 += 64) {
    const int dep = d0 + lane;
    int acc = 0;
    // unconditional clamped loads, masked arithmetically (get_pixel's white
    // off the mask/image), so the unrolled loads overlap
#pragma unroll 8
    for (int i = w; i < scan; i += kWaves) {
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
#pragma unroll
      for (int k = 0; k < kWaves; k++) B += part[k][lane];
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

template <int FMT>
static void launch_rot_t(const PlaneRef& img, const RotGeom& g, const RotTable* table,
                         const Rect* masks, const int32_t* mask_active, int mask_index,
                         int32_t* peaks, int count, hipStream_t st, int nangles, int max_scan,
                         const RotScratch& R, float max_abs_angle) {
  // Band columns: every left/right line lies within scan*tan(max |angle|)
  // columns of the mask edge (line_setup), plus the kDepth steps and the
  // truncation slack.  A wider band (k_rot_final re-checks) takes k_rot_line.
  const float tn = tanf(fminf(fabsf(max_abs_angle), 1.5f));
  const int band_cap =
      imin(kBandCapMax, (int)ceilf((float)imax(max_scan, 1) * tn) + kDepth + 4);
  const size_t band_lds = sizeof(uint16_t) * kSliceRows * (size_t)band_cap;
  allow_dynamic_lds((const void*)k_rot_band_g, band_lds);
  UPH_LAUNCH_DIAG(1, k_rot_band_g, dim3(rot_slices(max_scan), g.nedges, count),
                  dim3(kBandThreads), band_lds, st, img, g, table, masks, mask_active, count,
                  max_scan, R, (int)FMT, band_cap);
  const int nlines = count * g.nedges * nangles;
  UPH_LAUNCH_DIAG(128, k_rot_final, dim3((nlines + 3) / 4), dim3(256), 0, st, g, table, masks,
                  mask_active, mask_index, peaks, count, max_scan, R, band_cap);
  const size_t lds = sizeof(int32_t) * 2 * (size_t)(max_scan > 0 ? max_scan : 1);
  allow_dynamic_lds((const void*)k_rot_line<FMT>, lds);
  UPH_LAUNCH_DIAG(128, k_rot_line<FMT>, dim3(imin(nlines, 1024)), dim3(kWalkThreads), lds, st, img, g,
                  table, masks, mask_active, mask_index, peaks, count, max_scan, R);
}

void launch_rotation_peaks(const PlaneRef& img, const RotGeom& g, const RotTable* table,
                           const Rect* masks, const int32_t* mask_active, int mask_index,
                           int32_t* peaks, int count, hipStream_t st, int nangles,
                           int max_scan, int32_t* lines, float max_abs_angle) {
  if (g.nedges <= 0 || nangles <= 0) return;
  const int nlines = count * g.nedges * nangles;
  const RotScratch R = rot_scratch(lines, nlines, max_scan);
  // the launches below report a failure; column ranges start empty (0x7F.. / 0x80..)
  if (hipMemsetAsync(R.nlist, 0, sizeof(int32_t), st) != hipSuccess ||
      hipMemsetAsync(R.blo, 0x7F, sizeof(int32_t) * nlines, st) != hipSuccess ||
      hipMemsetAsync(R.bhi, 0x80, sizeof(int32_t) * nlines, st) != hipSuccess)
    return;
  UPH_LAUNCH_DIAG(16, k_rot_points, dim3((nlines + 255) / 256), dim3(256), 0, st, g, table, masks,
                  mask_active, count, R);
  switch (img.P.fmt) {
    case F_GRAY8:
      launch_rot_t<F_GRAY8>(img, g, table, masks, mask_active, mask_index, peaks, count, st,
                            nangles, max_scan, R, max_abs_angle);
      break;
    case F_Y400A:
      launch_rot_t<F_Y400A>(img, g, table, masks, mask_active, mask_index, peaks, count, st,
                            nangles, max_scan, R, max_abs_angle);
      break;
    default:
      launch_rot_t<F_RGB24>(img, g, table, masks, mask_active, mask_index, peaks, count, st,
                            nangles, max_scan, R, max_abs_angle);
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

const uint32_t* glibc_pow2_table(int* n) {
  static std::vector<uint32_t> table;
  static bool ok = false;
  static std::once_flag once;
  std::call_once(once, [] {
    static float (*volatile pw)(float, float) = powf;  // the process's glibc, not a fold
    glibc::build_pow2_table(pw, table);
    ok = true;
    for (uint32_t v : table) ok = ok && v != 0xffffffffu;
  });
  *n = (int)table.size();
  return ok ? table.data() : nullptr;
}

}  // namespace uph
